#!/bin/bash
# The automatic chunked visit order (cgx_abi.cpp build_sell, cgx_dist.cpp
# interior list): the GPU tests it touches (SELL forms, 512^3, march, value
# codes, the partitioned solves), 512^3 natural order against auto, and the
# 8-GPU slab floors. Stops at the first failing GPU step.
#   tools/gpu_order.sh TAG
set -o pipefail
TAG=${1:-order}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_bigsize.py \
    tests/test_gpu_march.py tests/test_gpu_value_codes.py tests/test_gpu_dist.py -m gpu -x -v \
    --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/gpu_order512.sh $TAG/p512 p3d_512 0 auto || exit 1
for o in 0 auto; do
  if [ "$o" = 0 ]; then export CGX_SELL_ORDER=0; else unset CGX_SELL_ORDER; fi
  timeout -k 10 300 python tools/slab_bench.py 3,256,256,32,2000 3,512,512,64,400 > $OUT/slab_$o.log 2>&1 || { echo "SLAB $o FAIL"; tail -20 $OUT/slab_$o.log; exit 1; }
  echo "slab order=$o"; grep -v amdgpu.ids $OUT/slab_$o.log | cut -c1-240
done
