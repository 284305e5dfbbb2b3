#!/bin/bash
# slab floors and 256^3: default (non-temporal vector streams) against a
# build without them (EXTRA=-DCGX_NO_STREAM_NT), interleaved
set -o pipefail
OUT=gpurun_out/${1:-slabnt}
mkdir -p $OUT
for rep in 1 2; do
  for lib in default build_ab/nont/libcgx.so; do
    tag=$(basename $(dirname $lib))_$rep
    ( [ "$lib" != default ] && export CGX_LIB=$lib; timeout -k 10 300 python tools/slab_bench.py 3,256,256,32,2000 3,128,128,128,1000 > $OUT/slab_$tag.log 2>&1 ) || { echo "SLAB $lib FAIL"; tail $OUT/slab_$tag.log; exit 1; }
    echo "[$lib r$rep]"; grep '^{' $OUT/slab_$tag.log | cut -c1-200
  done
done
