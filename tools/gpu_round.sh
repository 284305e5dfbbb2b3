#!/bin/bash
# GPU-box script: full gpu test-suite, smoke, dist checks (1 and 2 ranks on
# the box's GPU), short bench. Stops at the first failing GPU step.
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -rs > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -4 $OUT/pytest_gpu.log
[ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 200 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tests/dist_check.py > $OUT/dist1.log 2>&1 || { echo DIST1_FAIL; tail -20 $OUT/dist1.log; exit 1; }
grep world $OUT/dist1.log
timeout -k 10 200 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tests/dist_check.py > $OUT/dist2.log 2>&1; echo "dist2 rc=$?"
grep -E "world|rror|uplicate" $OUT/dist2.log | head -5
