#!/bin/bash
# GPU-box script: interleaved A/B of bench.py configurations, each given as
# "ENV=VAL,ENV2=VAL2|bench args" in $CFGS (';'-separated); ROUNDS rounds.
set -o pipefail
TAG=${1:-abcfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
IFS=';' read -ra LIST <<< "$CFGS"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for cfg in "${LIST[@]}"; do
    i=$((i+1))
    envs=${cfg%%|*}; args=${cfg#*|}
    ( [ -n "$envs" ] && export ${envs//,/ }; timeout -k 10 300 python bench.py --no-cpu $args > $OUT/b_${i}_r${r}.log 2>&1 ) || { echo "BENCH_FAIL [$cfg]"; tail $OUT/b_${i}_r${r}.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_${i}_r${r}.log').read().strip().splitlines()[-1]); ro=d['roofline']; print('[$cfg] r$r', d['value'], d['ms_per_step'], d['config'].get('spmv_variant'), ro['kernel'], ro['avg_us'], ro['other_kernels_avg_us'])"
  done
done
