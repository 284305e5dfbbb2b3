#!/bin/bash
# grid caps of the vector kernels for vectors under 8 M elements (the G3
# stand-in, the 256^3/8 slab): interleaved A/B of CGX_GRID_R_SMALL /
# CGX_GRID_P_SMALL
# (the CGX_GRID_*_SMALL knobs existed only in the A/B build of that run; the
# defaults won and the knobs were removed)
set -o pipefail
O=gpurun_out/${1:-smallgrid}
mkdir -p $O
for rep in 1 2; do
for rp in "256 512" "512 1024" "1024 1024" "128 256"; do
  set -- $rp
  CGX_GRID_R_SMALL=$1 CGX_GRID_P_SMALL=$2 timeout -k 10 200 python -u tools/slab_bench.py 3,256,256,32,2000 > $O/slab_$1_$2_$rep.log 2>&1 || { echo "slab failed"; tail $O/slab_$1_$2_$rep.log; exit 1; }
  CGX_GRID_R_SMALL=$1 CGX_GRID_P_SMALL=$2 timeout -k 10 200 python -u tools/configs_bench.py --configs g3_irr > $O/g3_$1_$2_$rep.log 2>&1 || { echo "g3 failed"; tail $O/g3_$1_$2_$rep.log; exit 1; }
  echo "R=$1 P=$2 slab $(grep '^{' $O/slab_$1_$2_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_body"], d["kernel_us"])') g3 $(grep '^{' $O/g3_$1_$2_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["it_per_s"], d["spmv_variant"])')"
done
done
