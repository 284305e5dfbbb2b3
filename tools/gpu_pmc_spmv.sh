#!/bin/bash
# GPU-box script: PMC counter passes over the SpMV(+p.Ap) kernel variants
# (tools/tune_spmv.py), one rocprofv3 run per counter group (--pmc with
# kernel dispatch only; no tracing domains). Outputs in gpurun_out/$TAG.
set -o pipefail
TAG=${1:-pmc}
VARIANTS=${VARIANTS:-15,31,63}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $GROUP -d $OUT/p$i -o run --output-format csv -- python3 tools/tune_spmv.py --configs 3d256 --variants $VARIANTS --rounds 1 --iters 3 > $OUT/p$i.log 2>&1 || { echo "PMC pass $i ($GROUP) failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $GROUP"
done <<EOF
${GROUPS_OVERRIDE:-GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS}
TA_TA_BUSY
TA_ADDR_STALLED_BY_TC_CYCLES
TA_DATA_STALLED_BY_TC_CYCLES
TD_TD_BUSY
TCP_PENDING_STALL_CYCLES
TCP_TCR_TCP_STALL_CYCLES
TCP_UTCL1_TRANSLATION_MISS
TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY
TCC_BUSY TCC_TAG_STALL
EOF
