#!/bin/bash
# value-code templates, round 2 of the A/B: tests, isolated (tune_spmv) and
# in-loop (bench, variant forced, interleaved) on 256^3, 4096^2, 512^3
set -o pipefail
TAG=${1:-vt3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "value_code or march or fdefer or sell or bigsize" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/tune_spmv.py --configs 3d256,2d4096 --variants 1875970,10264578,3973122,12361730 --rounds 5 > $OUT/tune.log 2>&1 || { echo TUNE_FAIL; tail -20 $OUT/tune.log; exit 1; }
cut -c1-130 $OUT/tune.log
b() {  # workload variant tag
  CGX_SPMV_VARIANT=$2 timeout -k 10 300 python bench.py --workload $1 --steps ${STEPS:-200} --warmup 10 --no-cpu --no-general --no-traffic > $OUT/b_$1_$2_$3.log 2>&1 || { echo "BENCH $1 $2 FAIL"; tail -20 $OUT/b_$1_$2_$3.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$1_$2_$3.log') if l.startswith('{')][-1]); r=d['roofline']; print('$1', $2, 'it/s', d['iterations_per_s'], 'spmv us', r['avg_us'], r['other_kernels_avg_us'])"
}
for rep in 1 2; do
  b p2d_4096 3973122 $rep && b p2d_4096 12361730 $rep || exit 1
  STEPS=40 b p3d_512 1613826 $rep && STEPS=40 b p3d_512 10264578 $rep || exit 1
done
for w in p3d_256 p2d_4096 p3d_512 p2d_128; do
  timeout -k 10 300 python bench.py --workload $w --steps 100 --warmup 10 --no-cpu --no-general --no-traffic > $OUT/auto_$w.log 2>&1 || { echo "AUTO $w FAIL"; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/auto_$w.log') if l.startswith('{')][-1]); print('auto $w', d['config']['spmv_variant'], d['iterations_per_s'])"
done
