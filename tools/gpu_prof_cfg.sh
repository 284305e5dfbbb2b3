#!/bin/bash
# rocprofv3 kernel-trace stats of tools/configs_bench.py for the given configs
# usage: gpu_prof_cfg.sh TAG CONFIGS
set -o pipefail
TAG=${1:-cfgprof}; CFGS=${2:-g3_irr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o cfg --output-format csv -- python3 tools/configs_bench.py --configs $CFGS > $OUT/cfg.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/cfg.log; exit 1; }
grep config $OUT/cfg.log
python3 - $OUT <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/prof/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print(f'{r["Name"][:90]:90s} {r["Calls"]:>6s} {float(r["AverageNs"])/1000:9.2f} us')
PY
