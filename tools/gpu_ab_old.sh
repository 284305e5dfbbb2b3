#!/bin/bash
# same-box A/B of the current tree's 1-GPU bench against an older build
# (build_ab/oldtree: that commit's bench.py, Python package and libcgx.so)
set -o pipefail
O=gpurun_out/${1:-abold}
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-general --steps 300 > $O/new_$rep.log 2>&1 || { echo "new failed"; tail -20 $O/new_$rep.log; exit 1; }
  tail -1 $O/new_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('new', d['iterations_per_s'], d['roofline']['avg_us'], d['roofline']['other_kernels_avg_us'])"
  (cd build_ab/oldtree && timeout -k 10 200 python -u bench.py --no-cpu --no-general --steps 300) > $O/old_$rep.log 2>&1 || { echo "old failed"; tail -20 $O/old_$rep.log; exit 1; }
  tail -1 $O/old_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('old', d['iterations_per_s'], d['roofline']['avg_us'], d['roofline']['other_kernels_avg_us'])"
done
