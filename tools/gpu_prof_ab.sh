#!/bin/bash
# rocprofv3 kernel stats of one config with the tree's libcgx and an A/B build
set -o pipefail
O=gpurun_out/${1:-profab}
ALT=${2}
CFG=${3:-p2d_128}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/base -o run --output-format csv -- python3 tools/configs_bench.py --configs $CFG > $O/base.log 2>&1 || { echo "base failed"; tail $O/base.log; exit 1; }
CGX_LIB=$ALT timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/alt -o run --output-format csv -- python3 tools/configs_bench.py --configs $CFG > $O/alt.log 2>&1 || { echo "alt failed"; tail $O/alt.log; exit 1; }
for w in base alt; do
  echo "== $w"
  f=$(find $O/$w -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$f')))[:8]:
    print(r['Name'][:90].replace('cgx::(anonymous namespace)::',''), r['Calls'], round(float(r['AverageNs'])/1e3,2))"
done
