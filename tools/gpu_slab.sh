#!/bin/bash
# Per-rank slab floors of the 8-GPU configs on one GPU, mode 3 (auto) against
# mode 4 (CGX_AUTO_FD=1), interleaved twice.
set -o pipefail
TAG=${1:-slab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for fd in 0 1; do
    CGX_AUTO_FD=$fd timeout -k 10 300 python tools/slab_bench.py 3,256,256,32,2000 3,512,512,64,400 > $OUT/slab_fd${fd}_$rep.log 2>&1 || { echo "SLAB fd=$fd FAIL"; tail -20 $OUT/slab_fd${fd}_$rep.log; exit 1; }
    cut -c1-220 $OUT/slab_fd${fd}_$rep.log
  done
done
