#!/bin/bash
# GPU-box script: gpu tests, then an interleaved A/B of the iteration modes
# (3 kernels vs fused) of bench.py on the same device.
set -o pipefail
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "Error|assert" $OUT/pytest_gpu.log | head -20; exit 1; }
for r in 1 2; do
  for m in 1 2; do
    timeout -k 10 300 python bench.py --no-cpu --mode $m > $OUT/bench_m${m}_r${r}.log 2>&1 || { echo BENCH_FAIL; tail $OUT/bench_m${m}_r${r}.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_m${m}_r${r}.log').read().strip().splitlines()[-1]); print('mode $m round $r', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_us'], d['roofline']['achieved'], d['roofline']['other_kernels_avg_us'])"
  done
done
