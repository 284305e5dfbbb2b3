#!/bin/bash
# GPU-box script for the round's measured record: full gpu test-suite, smoke,
# default bench (with the CPU baseline), rocprofv3 --kernel-trace --stats of
# the same bench command, then FETCH_SIZE and WRITE_SIZE PMC passes (separate
# runs, kernel dispatch counters only) of a short bench. Stops at the first
# failing GPU step. Outputs in gpurun_out/$TAG.
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --no-cpu > $OUT/bench_prof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_prof.log; exit 1; }
tail -1 $OUT/bench_prof.log
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C -d $OUT/pmc_$C -o run --output-format csv -- python3 bench.py --no-cpu --steps 10 --warmup 2 --profile-steps 0 > $OUT/pmc_$C.log 2>&1 || { echo "PMC $C FAIL"; tail -20 $OUT/pmc_$C.log; exit 1; }
  echo "pmc $C ok"
done
find $OUT -name "*stats*.csv" | head
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 --grid 64 --transport host --no-cpu > $OUT/bench_2rank_host.log 2>&1 || { echo DIST_BENCH_FAIL; tail -20 $OUT/bench_2rank_host.log; exit 1; }
grep metric $OUT/bench_2rank_host.log | cut -c1-300
timeout -k 10 600 python tools/configs_bench.py > $OUT/configs.log 2>&1 || { echo CONFIGS_FAIL; tail -20 $OUT/configs.log; exit 1; }
grep config $OUT/configs.log
