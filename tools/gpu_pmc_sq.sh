#!/bin/bash
# SQ/GRBM counter passes over the isolated production SpMV (tools/tune_spmv.py)
set -o pipefail
OUT=gpurun_out/${1:-pmcsq}
V=${2:-821250}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU" \
         "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TA_BUSY_max TA_TA_BUSY_sum TD_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python3 tools/tune_spmv.py --configs 3d256 --variants $V --rounds 1 --iters 5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
python3 tools/pmc_summary.py $OUT k_spmv_dot
