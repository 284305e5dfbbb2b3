#!/bin/bash
# GPU suite with mode 5 in the auto choice, smoke, the p2d_128 bench line.
set -o pipefail
TAG=${1:-coopf}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for w in p2d_128 g3_standin; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 2000 --warmup 50 --no-traffic > $OUT/bench_$w.log 2>&1 || { echo "BENCH $w FAIL"; tail -20 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log | cut -c1-900
done
