#!/bin/bash
# CSR-stream on 16-bit column deltas: tests, isolated SpMV A/B on the G3
# stand-in, the g3_standin bench line.
set -o pipefail
TAG=${1:-c16}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_col16.py tests/test_gpu_bigsize.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/tune_spmv.py --configs irr --variants 5,133,265,13,135 --rounds 5 --iters 20 > $OUT/tune.log 2>&1 || { echo TUNE_FAIL; tail $OUT/tune.log; exit 1; }
grep '^{' $OUT/tune.log | cut -c1-170
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --workload g3_standin --steps 2000 --warmup 50 --no-traffic --no-cpu --no-general > $OUT/bench_g3_$r.log 2>&1 || { echo BENCH_FAIL; tail $OUT/bench_g3_$r.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_g3_$r.log') if l.startswith('{')][-1]); r=d['roofline']; print('g3', d['iterations_per_s'], d['config']['spmv_variant'], r['avg_us'], r['frac'], r['other_kernels_avg_us'])"
done
