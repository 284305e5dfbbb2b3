#!/bin/bash
# interleaved bench A/B of the tree's libcgx against an A/B build ($2, loaded
# with CGX_LIB)
set -o pipefail
O=gpurun_out/${1:-ablib}
ALT=${2:-build_ab/pnt/libcgx.so}
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-general --steps 300 > $O/base_$rep.log 2>&1 || { echo "base failed"; tail -20 $O/base_$rep.log; exit 1; }
  tail -1 $O/base_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('base', d['iterations_per_s'], d['roofline']['avg_us'], d['roofline']['other_kernels_avg_us'])"
  CGX_LIB=$ALT timeout -k 10 200 python -u bench.py --no-cpu --no-general --steps 300 > $O/alt_$rep.log 2>&1 || { echo "alt failed"; tail -20 $O/alt_$rep.log; exit 1; }
  tail -1 $O/alt_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('alt ', d['iterations_per_s'], d['roofline']['avg_us'], d['roofline']['other_kernels_avg_us'])"
done
