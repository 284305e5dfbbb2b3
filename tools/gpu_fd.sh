#!/bin/bash
# mode 4 (fused deferred-x iteration): its GPU tests, then the bench at
# 256^3 and 4096^2 in modes 3 and 4 (interleaved), every step under a limit
set -o pipefail
O=gpurun_out/${1:-fd1}
mkdir -p $O
(while true; do date > $O/heartbeat; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 500 python -u -m pytest tests/test_gpu_fdefer.py tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed: $?"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for mode in 3 4; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-general --mode $mode > $O/bench_m${mode}_$rep.log 2>&1 || { echo "bench m$mode failed"; tail -20 $O/bench_m${mode}_$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_m${mode}_$rep.log').read().strip().splitlines()[-1]); print('m$mode', d['iterations_per_s'], d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['other_kernels_avg_us'])"
done
done
