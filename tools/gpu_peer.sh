#!/bin/bash
# peer transport on one GPU: the dist tests, then 2-rank bench rehearsals
# (host transport vs host setup + device peer iteration)
set -o pipefail
O=gpurun_out/${1:-peer}
mkdir -p $O
(while true; do date > $O/heartbeat; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 \
    --timeout-method thread > $O/pytest_dist.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_dist.log; exit 1; }
tail -3 $O/pytest_dist.log
for t in host-peer host; do
  timeout -k 10 300 python -u bench.py --gpus 2 --transport $t --steps 200 --warmup 10 \
      --no-cpu --profile-steps 20 > $O/bench2_$t.log 2>&1 || { echo "bench $t failed"; tail -30 $O/bench2_$t.log; exit 1; }
  tail -1 $O/bench2_$t.log | cut -c1-600
done
