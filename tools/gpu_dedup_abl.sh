#!/bin/bash
# timing ablation: every slice reads one shared code chunk (CGX_VC_DEDUP=2,
# wrong values: isolated SpMV timing only) against each slice its own
set -o pipefail
O=gpurun_out/${1:-dedupabl}
mkdir -p $O
tail -1 $O/pytest.log 2>/dev/null
for rep in 1 2; do
for d in 2 0; do
  CGX_VC_DEDUP=$d timeout -k 10 200 python -u tools/tune_spmv.py --configs 3d256 --variants 1875970 --rounds 3 --iters 20 > $O/tune_d${d}_$rep.log 2>&1 || { echo "tune d$d failed"; tail -20 $O/tune_d${d}_$rep.log; exit 1; }
  grep '^{' $O/tune_d${d}_$rep.log | cut -c1-200 | sed "s/^/d$d /"
done
done
