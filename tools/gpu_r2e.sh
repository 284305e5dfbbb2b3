#!/bin/bash
# round 2 step e: the current tree's whole GPU suite, smoke, the default bench,
# a rocprofv3 kernel-trace of the bench and the FETCH/WRITE PMC passes (one
# counter group per run); every GPU step under its own limit
set -o pipefail
O=gpurun_out/${1:-r2e}
mkdir -p $O
(while true; do date > $O/heartbeat; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
timeout -k 10 240 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --no-cpu --no-general --steps 100 \
    > $O/prof_bench.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof_bench.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $O/bench_kernel_stats.csv
head -6 $O/bench_kernel_stats.csv | cut -c1-200
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc_$C -o run --output-format csv -- python3 bench.py --no-cpu --no-general --steps 10 --warmup 2 --profile-steps 0 > $O/pmc_$C.log 2>&1 || { echo "PMC $C FAIL"; tail -20 $O/pmc_$C.log; exit 1; }
  echo "pmc $C ok"
done
