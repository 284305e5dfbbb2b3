#!/bin/bash
# halo push merged into the interior SpMV launch and the all-reduces into
# their consumer kernels (both on / both off): the dist GPU tests, then
# the 2-rank one-GPU rehearsal of the peer path (host setup + peer iteration)
# with the merge on and off (interleaved), and the 1-GPU bench (no change
# expected: the single-device SpMV only gained the wg0 = 0 offset)
set -o pipefail
O=gpurun_out/${1:-pushmerge}
mkdir -p $O
(while true; do date > $O/heartbeat; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 500 --timeout-method thread \
    > $O/pytest_dist.log 2>&1 || { echo "pytest failed: $?"; tail -40 $O/pytest_dist.log; exit 1; }
tail -1 $O/pytest_dist.log
for rep in 1 2; do
for cfg in "1 1" "1 0" "0 0"; do
  set -- $cfg
  CGX_PEER_AR_FUSE=$1 CGX_PEER_PUSH_MERGE=$1 CGX_PEER_WAIT_FOLD=$2 timeout -k 10 240 python -u bench.py --gpus 2 --transport host-peer --no-cpu --no-general --steps 300 --profile-steps 0 > $O/bench2_m$1_f$2_$rep.log 2>&1 || { echo "bench2 $cfg failed"; tail -20 $O/bench2_m$1_f$2_$rep.log; exit 1; }
  grep '^{' $O/bench2_m$1_f$2_$rep.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('merge+fuse', '$1', 'fold', '$2', d['n_gpus'], d['iterations_per_s'])"
done
done
timeout -k 10 240 python -u bench.py --no-cpu --no-general --steps 300 > $O/bench1.log 2>&1 || { echo "bench1 failed"; tail -20 $O/bench1.log; exit 1; }
tail -1 $O/bench1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('1gpu', d['iterations_per_s'], d['roofline']['avg_us'])"
