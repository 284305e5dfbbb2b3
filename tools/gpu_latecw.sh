#!/bin/bash
# late code-word load (variant bit 4194304) against the production stencil
# form: isolated SpMV A/B, then the bench with each forced (interleaved)
set -o pipefail
O=gpurun_out/${1:-latecw}
mkdir -p $O
timeout -k 10 300 python -u tools/tune_spmv.py --configs 3d256,2d4096 --variants 1875970,6070274,1613826,5808130 \
    --rounds 3 --iters 10 > $O/tune.log 2>&1 || { echo "tune failed"; tail -20 $O/tune.log; exit 1; }
cut -c1-250 $O/tune.log
for rep in 1 2; do
for v in 1875970 6070274; do
  CGX_SPMV_VARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu --no-general --steps 300 > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.log; exit 1; }
  tail -1 $O/bench_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($v, d['iterations_per_s'], d['roofline']['avg_us'], d['roofline']['other_kernels_avg_us'], d['config']['spmv_variant'])"
done
done
