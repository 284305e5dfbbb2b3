#!/bin/bash
# GPU tests on the in-tree libcgx.so (unless SKIP_TESTS), then isolated
# SpMV timings and an interleaved in-loop bench A/B against the libraries in
# $LIBS (loaded through CGX_LIB).
#   LIBS="build/ab/a.so build/ab/b.so" bash tools/gpu_lib_ab.sh TAG [variants]
set -o pipefail
OUT=gpurun_out/${1:-libab}
V=${2:-821250}
LIBS=${LIBS:-build/ab/libcgx_base.so}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_value_codes.py tests/test_gpu_sell.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for L in default $LIBS; do
  if [ "$L" = default ]; then unset CGX_LIB; else export CGX_LIB=$L; fi
  timeout -k 10 300 python tools/tune_spmv.py --configs 3d256,2d4096 --variants $V > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
  echo "== $L"; grep config $OUT/tune.log | cut -c1-120
done
for r in 1 2; do
  for L in default $LIBS; do
    if [ "$L" = default ]; then unset CGX_LIB; else export CGX_LIB=$L; fi
    timeout -k 10 300 python bench.py --no-cpu $BENCH_ARGS > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
    echo "[$L r$r] $(tail -1 $OUT/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["iterations_per_s"], d["config"]["spmv_variant"], r["avg_us"], r["other_kernels_avg_us"])')"
  done
done
