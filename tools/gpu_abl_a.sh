#!/bin/bash
# timing ablation: the 3-D stencil slices' +-a gathers read the wave's own
# center lines (variant 6070274, wrong values) against the production form
set -o pipefail
O=gpurun_out/${1:-abla}
mkdir -p $O
timeout -k 10 300 python -u tools/tune_spmv.py --configs 3d256 --variants 1875970,6070274 --rounds 5 --iters 20 > $O/tune.log 2>&1 || { echo "tune failed"; tail -20 $O/tune.log; exit 1; }
grep '^{' $O/tune.log | cut -c1-220
