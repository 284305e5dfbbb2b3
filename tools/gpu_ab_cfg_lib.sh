#!/bin/bash
# interleaved configs_bench A/B of the tree's libcgx against an A/B build
set -o pipefail
O=gpurun_out/${1:-abcfg}
ALT=${2}
CFG=${3:-p2d_4096}
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 200 python -u tools/configs_bench.py --configs $CFG > $O/base_$rep.log 2>&1 || { echo "base failed"; tail $O/base_$rep.log; exit 1; }
  echo "base $(grep '^{' $O/base_$rep.log | cut -c1-160)"
  CGX_LIB=$ALT timeout -k 10 200 python -u tools/configs_bench.py --configs $CFG > $O/alt_$rep.log 2>&1 || { echo "alt failed"; tail $O/alt_$rep.log; exit 1; }
  echo "alt  $(grep '^{' $O/alt_$rep.log | cut -c1-160)"
done
