#!/bin/bash
# GPU-box script: SpMV variant A/B, then rocprofv3 kernel-trace and PMC passes
# of a short bench.py run. Every GPU step has its own time limit; the script
# stops at the first failure. Outputs under gpurun_out/$TAG.
set -o pipefail
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${SKIP_TUNE:-0}" != "1" ]; then
  timeout -k 10 300 python tools/tune_spmv.py ${TUNE_ARGS:-} > $OUT/tune.log 2>&1 || { echo TUNE_FAIL; tail -20 $OUT/tune.log; exit 1; }
  grep config $OUT/tune.log
fi
BENCH="bench.py --steps 50 --warmup 5 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $BENCH > $OUT/bench_trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $OUT/bench_trace.log; exit 1; }
tail -1 $OUT/bench_trace.log
PBENCH="bench.py --steps 10 --warmup 2 --no-cpu --profile-steps 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 $PBENCH > $OUT/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAIL; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 $PBENCH > $OUT/pmc_write.log 2>&1 || { echo PMC_WRITE_FAIL; tail -20 $OUT/pmc_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_hit -o run --output-format csv -- python3 $PBENCH > $OUT/pmc_hit.log 2>&1 || { echo PMC_HIT_FAIL; tail -20 $OUT/pmc_hit.log; exit 1; }
find $OUT -name "*.csv" | head -30
