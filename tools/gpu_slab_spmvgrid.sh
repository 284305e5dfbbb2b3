#!/bin/bash
# SpMV grid on the 256^3/8 slab (CGX_SPMV_GRID, A/B only): does a smaller
# persistent grid (more slices per wave) cut the small matrix's fixed cost?
set -o pipefail
O=gpurun_out/${1:-slabgrid}
mkdir -p $O
for rep in 1 2; do
for g in 0 640 960 1536; do
  if [ $g = 0 ]; then unset CGX_SPMV_GRID; else export CGX_SPMV_GRID=$g; fi
  timeout -k 10 200 python -u tools/slab_bench.py 3,256,256,32,2000 > $O/slab_$g_$rep.log 2>&1 || { echo "slab failed"; tail $O/slab_$g_$rep.log; exit 1; }
  echo "grid $g $(grep '^{' $O/slab_$g_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_body"], d["spmv_variant"], d["kernel_us"])')"
done
done
