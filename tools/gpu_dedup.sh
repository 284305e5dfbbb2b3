#!/bin/bash
# value-code chunk sharing (CGX_VC_SHARE): correctness tests, the isolated
# SpMV and the bench with sharing on / off interleaved
set -o pipefail
O=gpurun_out/${1:-share}
mkdir -p $O
(while true; do date > $O/heartbeat; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
for c in 64 256; do
for d in 1 0; do
  CGX_VC_SHARE_COPIES=$c CGX_VC_SHARE=$d timeout -k 10 200 python -u tools/tune_spmv.py --configs 3d256,2d4096 --variants 1875970,1613826 --rounds 3 --iters 20 > $O/tune_s$d.log 2>&1 || { echo "tune s$d failed"; tail -20 $O/tune_s$d.log; exit 1; }
  grep '^{' $O/tune_s$d.log | cut -c1-200 | sed "s/^/c$c s$d /"
done
done
for rep in 1 2; do
for cfg in "1 64" "1 1024" "0 64"; do
  set -- $cfg
  CGX_VC_SHARE=$1 CGX_VC_SHARE_COPIES=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-general --steps 300 > $O/bench_s$1_c$2_$rep.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_s$1_c$2_$rep.log; exit 1; }
  tail -1 $O/bench_s$1_c$2_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('share', '$1', 'copies', '$2', d['iterations_per_s'], r['avg_us'], r['bytes_per_launch'], r['other_kernels_avg_us'])"
done
done
