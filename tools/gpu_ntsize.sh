#!/bin/bash
# size-dependent non-temporal vector streams: slabs, G3 stand-in, 256^3, tests
set -o pipefail
OUT=gpurun_out/${1:-ntsize}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fdefer.py tests/test_gpu_fullsize.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/slab_bench.py 3,256,256,32,2000 3,128,128,128,1000 > $OUT/slab.log 2>&1 || { echo SLAB_FAIL; tail $OUT/slab.log; exit 1; }
grep '^{' $OUT/slab.log | cut -c1-200
for w in g3_standin p3d_256; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 400 --warmup 20 --no-traffic --no-cpu --no-general > $OUT/bench_$w.log 2>&1 || { echo "BENCH $w FAIL"; tail $OUT/bench_$w.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_$w.log') if l.startswith('{')][-1]); r=d['roofline']; print('$w', d['iterations_per_s'], d['config']['spmv_variant'], r['avg_us'], r['other_kernels_avg_us'])"
done
