#!/bin/bash
# round 2 record run: GPU suite, smoke, default bench (with CPU baseline and
# csr_general), rocprofv3 kernel-trace of the bench, FETCH/WRITE PMC passes,
# all configs in auto mode, the per-rank slab of 256^3/8 on one GPU, and the
# 2-rank one-GPU rehearsal of the peer path; every GPU step under a limit
set -o pipefail
O=gpurun_out/${1:-r2h}
mkdir -p $O
(while true; do date > $O/heartbeat; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --no-cpu --no-general --steps 100 \
    > $O/prof_bench.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof_bench.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $O/bench_kernel_stats.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc_$C -o run --output-format csv -- python3 bench.py --no-cpu --no-general --steps 10 --warmup 2 --profile-steps 0 > $O/pmc_$C.log 2>&1 || { echo "PMC $C FAIL"; tail -20 $O/pmc_$C.log; exit 1; }
done
timeout -k 10 400 python -u tools/configs_bench.py > $O/configs.log 2>&1 || { echo "configs failed"; tail -20 $O/configs.log; exit 1; }
grep '^{' $O/configs.log | cut -c1-200
timeout -k 10 300 python -u tools/slab_bench.py > $O/slab.log 2>&1 || { echo "slab failed"; tail -20 $O/slab.log; exit 1; }
grep '^{' $O/slab.log | cut -c1-300
timeout -k 10 300 python -u bench.py --gpus 2 --transport host-peer --no-cpu --no-general --steps 300 > $O/bench_2rank_hostpeer.log 2>&1 || { echo "2rank failed"; tail -20 $O/bench_2rank_hostpeer.log; exit 1; }
grep '^{' $O/bench_2rank_hostpeer.log | tail -1 | cut -c1-300
