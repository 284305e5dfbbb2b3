#!/bin/bash
# GPU-box script: gpu tests on the default libcgx.so, then an interleaved A/B
# of bench.py between the default build and the builds named in $LIBS
# (space-separated .so paths, loaded through CGX_LIB).
set -o pipefail
TAG=${1:-ablib}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -3 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "Error|assert" $OUT/pytest_gpu.log | head -20; exit 1; }
fi
for r in 1 2; do
  i=0
  for L in default $LIBS; do
    i=$((i+1))
    if [ "$L" = default ]; then unset CGX_LIB; else export CGX_LIB=$L; fi
    timeout -k 10 300 python bench.py --no-cpu $BENCH_ARGS > $OUT/bench_${i}_r${r}.log 2>&1 || { echo BENCH_FAIL $L; tail $OUT/bench_${i}_r${r}.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_${i}_r${r}.log').read().strip().splitlines()[-1]); print('$L round $r', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_us'], d['roofline']['other_kernels_avg_us'])"
  done
done
