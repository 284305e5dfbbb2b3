#!/bin/bash
# GPU-box script: interleaved A/B of tools/configs_bench.py under environment
# settings. $ENVS: ';'-separated "ENV=VAL,ENV2=VAL2" entries ("-" = none);
# $CONFIGS: configs_bench --configs list; ROUNDS rounds.
set -o pipefail
TAG=${1:-abconf}
OUT=gpurun_out/$TAG
mkdir -p $OUT
IFS=';' read -ra LIST <<< "$ENVS"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for envs in "${LIST[@]}"; do
    i=$((i+1))
    ( [ "$envs" != "-" ] && export ${envs//,/ }; timeout -k 10 300 python tools/configs_bench.py --configs ${CONFIGS:-g3_irr} > $OUT/c_${i}_r${r}.log 2>&1 ) || { echo "CFG_FAIL [$envs]"; tail $OUT/c_${i}_r${r}.log; exit 1; }
    grep config $OUT/c_${i}_r${r}.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('[$envs] r$r', d['config'], d['it_per_s'], d['ms_per_iter'], d['frac_of_8TBps'], d['spmv_variant'])"
  done
done
