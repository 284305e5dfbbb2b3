#!/bin/bash
# GPU-box script: default bench (with CPU baseline), an A/B of the timed
# region without per-kernel events, a rocprofv3 --kernel-trace --stats run of
# the default bench command, and a 2-rank rehearsal of the N>1 bench path on
# one GPU (host transport; numbers meaningless). Outputs in gpurun_out/$TAG.
set -o pipefail
TAG=${1:-bench}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log
timeout -k 10 300 python bench.py --no-cpu --profile-steps 0 > $OUT/bench_nokt.log 2>&1 || { echo BENCH2_FAIL; tail -20 $OUT/bench_nokt.log; exit 1; }
tail -1 $OUT/bench_nokt.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --no-cpu > $OUT/bench_prof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_prof.log; exit 1; }
tail -1 $OUT/bench_prof.log
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 --grid 64 --transport host > $OUT/bench_2rank_host.log 2>&1 || { echo DIST_BENCH_FAIL; tail -20 $OUT/bench_2rank_host.log; exit 1; }
grep metric $OUT/bench_2rank_host.log
find $OUT -name "*stats*.csv"
