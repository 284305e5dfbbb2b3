#!/bin/bash
# round 2 step d: whole GPU suite, the default bench, the configs sweep, and a
# rocprofv3 kernel-trace of the bench; every GPU step under its own limit
set -o pipefail
O=gpurun_out/${1:-r2d}
mkdir -p $O
(while true; do date > $O/heartbeat; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 240 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 400 python -u tools/configs_bench.py > $O/configs.log 2>&1 || { echo "configs failed"; tail -20 $O/configs.log; exit 1; }
grep '^{' $O/configs.log | cut -c1-260
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --no-cpu --no-general --steps 100 \
    > $O/prof_bench.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof_bench.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $O/bench_kernel_stats.csv
head -6 $O/bench_kernel_stats.csv | cut -c1-200
