#!/bin/bash
# rocprofv3 --kernel-trace --stats of the per-config bench lines whose
# dominant kernel changed this round (mode 5 at 128^2, CSR on 16-bit column
# deltas on the G3 stand-in)
set -o pipefail
OUT=gpurun_out/${1:-cfgprof}
mkdir -p $OUT
export TMPDIR=/tmp
for w in p2d_128 g3_standin; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 2000 --warmup 50 --no-cpu --no-general --no-traffic > $OUT/bench_$w.log 2>&1 || { echo "PROF $w FAIL"; tail $OUT/bench_$w.log; exit 1; }
  f=$(find $OUT/prof_$w -name "*kernel_stats.csv" | head -1)
  cp $f $OUT/${w}_kernel_stats.csv
  python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/${w}_kernel_stats.csv')))[:6]: print('$w', r['Name'][:70], r['Calls'], r['AverageNs'])"
done
