#!/bin/bash
# Per-rank slab floors of the 8-GPU configs on one GPU, modes 3, 4 and 6
# (MODES overrides), interleaved twice.
set -o pipefail
TAG=${1:-slab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for m in ${MODES:-3 4 6}; do
    timeout -k 10 300 python tools/slab_bench.py --mode $m 3,256,256,32,2000 3,512,512,64,400 > $OUT/slab_m${m}_$rep.log 2>&1 || { echo "SLAB mode $m FAIL"; tail -20 $OUT/slab_m${m}_$rep.log; exit 1; }
    cut -c1-220 $OUT/slab_m${m}_$rep.log
  done
done
