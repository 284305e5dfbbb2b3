#!/bin/bash
# vector-kernel grid sizes on cache-resident sizes (slab floor, G3 stand-in)
# and 256^3: default build against the libraries in $LIBS, interleaved
set -o pipefail
OUT=gpurun_out/${1:-gridab}
mkdir -p $OUT
for rep in 1 2; do
  for lib in default $LIBS; do
    t=$(basename $(dirname $lib))_$rep
    ( [ "$lib" != default ] && export CGX_LIB=$lib
      timeout -k 10 300 python tools/slab_bench.py 3,256,256,32,2000 > $OUT/slab_$t.log 2>&1 &&
      timeout -k 10 300 python bench.py --workload g3_standin --steps 2000 --warmup 50 --no-cpu --no-general --no-traffic > $OUT/g3_$t.log 2>&1 &&
      timeout -k 10 300 python bench.py --steps 400 --warmup 20 --no-cpu --no-general --no-traffic > $OUT/p3_$t.log 2>&1 ) || { echo "FAIL $lib"; exit 1; }
    echo "[$lib r$rep] slab $(grep '^{' $OUT/slab_$t.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["us_per_body"])') us/body; g3 $(grep '^{' $OUT/g3_$t.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["iterations_per_s"])') it/s; 256^3 $(grep '^{' $OUT/p3_$t.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["iterations_per_s"])') it/s"
  done
done
