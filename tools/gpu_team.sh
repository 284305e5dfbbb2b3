#!/bin/bash
# team walk (variant bit 4194304): isolated SpMV A/B with the bit-exactness
# check against the production form, then the bench with each forced
set -o pipefail
O=gpurun_out/${1:-team}
mkdir -p $O
timeout -k 10 300 python -u tools/tune_spmv.py --configs 3d256,3d128 --variants 1875970,6070274 --rounds 5 --iters 20 > $O/tune.log 2>&1 || { echo "tune failed"; tail -20 $O/tune.log; exit 1; }
grep '^{' $O/tune.log | cut -c1-220
for rep in 1 2; do
for v in 6070274 1875970; do
  CGX_SPMV_VARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu --no-general --steps 300 > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.log; exit 1; }
  tail -1 $O/bench_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($v, d['iterations_per_s'], d['roofline']['avg_us'], d['roofline']['other_kernels_avg_us'], d['config']['spmv_variant'])"
done
done
