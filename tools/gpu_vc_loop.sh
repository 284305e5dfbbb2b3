#!/bin/bash
# value-code SpMV: GPU tests touching the SpMV grid, isolated A/B, in-loop
# bench A/B (resident grid cap on/off, value codes off)
set -o pipefail
OUT=gpurun_out/${1:-vcloop}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_value_codes.py tests/test_gpu_sell.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/tune_spmv.py --configs 3d256 --variants 296962,821250,559106,821266 > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep config $OUT/tune.log | cut -c1-130
for cfg in "" "CGX_SPMV_VARIANT=296962" "CGX_SPMV_VARIANT=821250"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  echo "[$cfg] $(tail -1 $OUT/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["iterations_per_s"], d["config"]["spmv_variant"], r["avg_us"], r["other_kernels_avg_us"])')"
done
