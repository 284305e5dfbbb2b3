#!/bin/bash
# plane-march SpMV: its GPU tests, the isolated A/B against the stencil form,
# then the bench with each form forced (in-loop SpMV time) and the default
set -o pipefail
O=gpurun_out/${1:-march}
mkdir -p $O
(while true; do date > $O/heartbeat; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_march.py -x -v --timeout 120 \
    --timeout-method thread > $O/pytest_march.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_march.log; exit 1; }
tail -2 $O/pytest_march.log
timeout -k 10 300 python -u tools/tune_spmv.py --configs 3d256,2d4096 --variants 1875970,3973122,1613826,3710978 \
    --rounds 3 --iters 10 > $O/tune.log 2>&1 || { echo "tune failed"; tail -20 $O/tune.log; exit 1; }
cut -c1-300 $O/tune.log
for v in 1875970 3973122; do
  CGX_SPMV_VARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu --no-general --steps 300 > $O/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 1; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($v, d['iterations_per_s'], d['roofline']['avg_us'], d['roofline']['other_kernels_avg_us'], d['config']['spmv_variant'])"
done
timeout -k 10 200 python -u bench.py --no-cpu --steps 300 > $O/bench_default.log 2>&1 || { echo "bench default failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-900
