#!/bin/bash
# PMC passes over the isolated SpMV (tools/tune_spmv.py), stencil form vs
# plane march, one rocprofv3 run per counter group (kernel dispatch only)
set -o pipefail
O=gpurun_out/${1:-pmcmarch}
CFG=${CFG:-3d256}
VARS=${VARS:-1875970,3973122}
mkdir -p $O
export TMPDIR=/tmp
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $GROUP -d $O/p$i -o run --output-format csv -- \
      python3 tools/tune_spmv.py --configs $CFG --variants $VARS --rounds 1 --iters 3 \
      > $O/p$i.log 2>&1 || { echo "PMC pass $i ($GROUP) failed"; tail -5 $O/p$i.log; exit 1; }
  echo "pass $i ok: $GROUP"
done <<EOF
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum
TD_TD_BUSY_sum TD_BUSY_max
EOF
python3 tools/pmc_summary.py $O k_spmv_dot | tee $O/summary.txt
