#!/bin/bash
# isolated SpMV A/B of the plane march under grid / run-length settings
# (each setting is read once per process: one tune run per setting).
# SETTINGS: ';'-separated "tag [VAR=value ...]" entries
set -o pipefail
O=gpurun_out/${1:-marchenv}
CFG=${CFG:-3d256}
VARS=${VARS:-1875970,3973122}
SETTINGS=${SETTINGS:-"base;grid512 CGX_SPMV_GRID=512;len8 CGX_MARCH_LEN=8"}
mkdir -p $O
IFS=';' read -ra LIST <<< "$SETTINGS"
for setting in "${LIST[@]}"; do
  read -ra W <<< "$setting"
  tag=${W[0]}
  env "${W[@]:1}" DUMMY=1 timeout -k 10 150 python -u tools/tune_spmv.py --configs $CFG \
      --variants $VARS --rounds 3 --iters 10 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  grep '"variant"' $O/$tag.log | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$tag', d['config'], d['variant'], d['median_us'], d['bitexact_vs_v0'])"
done
