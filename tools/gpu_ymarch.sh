#!/bin/bash
# y-march (kYM) against the consecutive walk and the z-march at 256^3: time,
# bit-exactness (tune_spmv), run lengths, FETCH
set -o pipefail
OUT=gpurun_out/${1:-ym}
mkdir -p $OUT
export TMPDIR=/tmp
V=10264578,29138946,20750338,12361730
timeout -k 10 300 python tools/tune_spmv.py --configs 3d256 --variants $V --rounds 4 --iters 10 > $OUT/tune.log 2>&1 || { echo TUNE_FAIL; tail -20 $OUT/tune.log; exit 1; }
grep '^{' $OUT/tune.log | cut -c1-190
for L in 4 8 16 64; do
  CGX_MARCH_LEN=$L timeout -k 10 200 python tools/tune_spmv.py --configs 3d256 --variants 10264578,29138946 --rounds 3 --iters 10 > $OUT/tune_L$L.log 2>&1 || { echo "TUNE L$L FAIL"; tail $OUT/tune_L$L.log; exit 1; }
  echo "L=$L"; grep '^{' $OUT/tune_L$L.log | cut -c1-150
done
