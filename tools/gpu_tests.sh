#!/bin/bash
# GPU test suite + smoke + the driver's bench command (no profiles).
#   tools/gpu_tests.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-t}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
K=${2:+-k "$2"}
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread $K \
    > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-traffic > $OUT/bench_driver.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench_driver.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/bench_driver.log') if l.startswith('{')][-1]); r=d['roofline']; print('it/s', d['iterations_per_s'], 'spmv us', r['avg_us'], 'frac', r['frac'], r['other_kernels_avg_us'], {k: (v.get('iterations_per_s'), v.get('spmv_frac')) for k, v in (d.get('csr_general') or {}).items()})"
