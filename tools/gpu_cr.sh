#!/bin/bash
# Lane-shift (+-1 neighbours from adjacent lanes) value-code SpMV: GPU tests,
# isolated A/B, in-loop bench A/B against the plain pipelined form
set -o pipefail
OUT=gpurun_out/${1:-cr}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_value_codes.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/tune_spmv.py --configs 3d256,2d4096 --variants 821250,1869826,559106,1607682 > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep config $OUT/tune.log | cut -c1-150
for r in 1 2; do
for cfg in "CGX_SPMV_VARIANT=821250" "CGX_SPMV_VARIANT=1869826" "CGX_X=0"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  echo "[$cfg r$r] $(tail -1 $OUT/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["iterations_per_s"], d["config"]["spmv_variant"], r["avg_us"], r["other_kernels_avg_us"])')"
done
done
