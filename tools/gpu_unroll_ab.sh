#!/bin/bash
# Interleaved A/B of alternative library builds (CGX_LIB) on the driver's
# bench (256^3), the G3 stand-in and the 256x256x32 slab, two rounds.
#   bash tools/gpu_unroll_ab.sh TAG build/ab/x/libcgx.so ...
set -o pipefail
OUT=gpurun_out/${1:-unrollab}
shift
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for L in default "$@"; do
    if [ "$L" = default ]; then unset CGX_LIB; else export CGX_LIB=$L; fi
    for W in p3d_256 g3_standin; do
      timeout -k 10 300 python bench.py --no-cpu --no-general --no-traffic --workload $W > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
      echo "[$L $W r$r] $(tail -1 $OUT/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["iterations_per_s"], r["avg_us"], r["other_kernels_avg_us"])')"
    done
    timeout -k 10 300 python tools/slab_bench.py 3,256,256,32,2000 > $OUT/slab.log 2>&1 || { tail -20 $OUT/slab.log; exit 1; }
    echo "[$L slab r$r] $(cut -c1-200 $OUT/slab.log | tail -2)"
  done
done
