#!/bin/bash
# value-code templates: GPU tests of the value-code / march / fdefer / sell
# forms, isolated SpMV A/B (tune_spmv, interleaved), in-loop A/B (bench with
# the variant forced, interleaved twice).
set -o pipefail
TAG=${1:-vt}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "value_code_templates or march or fdefer or sell or bigsize" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/tune_spmv.py --configs 3d256,2d4096 --variants 1875970,10264578,3973122,12361730 --rounds 5 > $OUT/tune.log 2>&1 || { echo TUNE_FAIL; tail -20 $OUT/tune.log; exit 1; }
cut -c1-160 $OUT/tune.log
timeout -k 10 300 python tools/tune_spmv.py --configs 3d256,irr --variants 15,143,13,141,5 --rounds 5 > $OUT/tune_csr.log 2>&1 || { echo TUNE_CSR_FAIL; tail -20 $OUT/tune_csr.log; exit 1; }
cut -c1-160 $OUT/tune_csr.log
for rep in 1 2; do
  for v in 1875970 10264578; do
    CGX_SPMV_VARIANT=$v timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-general --no-traffic > $OUT/bench_${v}_$rep.log 2>&1 || { echo "BENCH $v FAIL"; tail -20 $OUT/bench_${v}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_${v}_$rep.log') if l.startswith('{')][-1]); r=d['roofline']; print($v, 'it/s', d['iterations_per_s'], 'spmv us', r['avg_us'], 'frac', r['frac'], r['other_kernels_avg_us'])"
  done
done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-general --no-traffic > $OUT/bench_auto.log 2>&1 || { echo "BENCH auto FAIL"; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_auto.log') if l.startswith('{')][-1]); print('auto', d['config']['spmv_variant'], d['iterations_per_s'])"
for rep in 1 2; do
  for v in 3973122 12361730; do
    CGX_SPMV_VARIANT=$v timeout -k 10 300 python bench.py --workload p2d_4096 --steps 200 --warmup 20 --no-cpu --no-general --no-traffic > $OUT/bench2d_${v}_$rep.log 2>&1 || { echo "BENCH2D $v FAIL"; tail -20 $OUT/bench2d_${v}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/bench2d_${v}_$rep.log') if l.startswith('{')][-1]); r=d['roofline']; print('2d', $v, 'it/s', d['iterations_per_s'], 'spmv us', r['avg_us'], r['other_kernels_avg_us'])"
  done
done
