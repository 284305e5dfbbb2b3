#!/bin/bash
# 256^3 in the loop: the autotune's SpMV form against the 8-bit (1613826) and
# streamed 4-bit (1875970) stencil forms forced by $CGX_SPMV_VARIANT, 400
# bodies each, interleaved twice; then the 20-body driver line three times.
#   tools/gpu_ab_codes.sh TAG
set -o pipefail
TAG=${1:-abc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in 0 1613826 1875970; do
    if [ $v = 0 ]; then unset CGX_SPMV_VARIANT; else export CGX_SPMV_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --workload p3d_256 --steps 400 --warmup 20 --profile-steps 50 \
        --no-cpu --no-general --no-traffic > $OUT/v${v}_$rep.log 2>&1 || { echo "FAIL v=$v"; tail -20 $OUT/v${v}_$rep.log; exit 1; }
    echo "v=$v $(grep -o '"iterations_per_s": [0-9.]*' $OUT/v${v}_$rep.log) $(grep -o '"spmv_variant": [0-9]*' $OUT/v${v}_$rep.log) $(grep -o '"avg_us": [0-9.]*' $OUT/v${v}_$rep.log)"
  done
done
unset CGX_SPMV_VARIANT
for rep in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-general --no-traffic \
      > $OUT/d20_$rep.log 2>&1 || { echo "FAIL d20"; tail -20 $OUT/d20_$rep.log; exit 1; }
  echo "driver 20: $(grep -o '"iterations_per_s": [0-9.]*' $OUT/d20_$rep.log)"
done
