#!/bin/bash
# GPU-box script: full gpu test-suite, then the setup-path timings.
set -o pipefail
TAG=${1:-setup}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAIL" $OUT/pytest_gpu.log | head -30; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 400 python tools/setup_bench.py > $OUT/setup.log 2>&1 || { echo SETUP_FAIL; tail -20 $OUT/setup.log; exit 1; }
tail -1 $OUT/setup.log
