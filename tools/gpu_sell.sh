#!/bin/bash
# GPU-box script: SELL tests + all gpu tests, SpMV variant A/B incl. SELL,
# then bench (default autotune) twice.
set -o pipefail
TAG=${1:-sell}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_sell.py -q -x > $OUT/pytest_sell.log 2>&1; rc=$?
tail -3 $OUT/pytest_sell.log
[ $rc -eq 0 ] || { echo "sell pytest rc=$rc"; grep -E "Error|assert|FAIL" $OUT/pytest_sell.log | head -30; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "Error|assert|FAIL" $OUT/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 400 python tools/tune_spmv.py --configs ${CONFIGS:-3d256,2d4096} --variants ${VARIANTS:-13,15,2048,2050,2064,31} --rounds 3 > $OUT/tune.log 2>&1 || { echo TUNE_FAIL; tail $OUT/tune.log; exit 1; }
grep config $OUT/tune.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu > $OUT/bench_r$r.log 2>&1 || { echo BENCH_FAIL; tail $OUT/bench_r$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_r$r.log').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['config'].get('spmv_variant'), d['roofline']['kernel'], d['roofline']['avg_us'], d['roofline']['other_kernels_avg_us'])"
done
