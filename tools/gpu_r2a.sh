#!/bin/bash
# round 2, step a: the whole GPU suite, then the bench (default) and a 2-rank
# host-transport bench rehearsal; every GPU step under its own time limit.
set -o pipefail
O=gpurun_out/${1:-r2a}
mkdir -p $O
(while true; do date > $O/heartbeat; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 240 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
