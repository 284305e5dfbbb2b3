#!/bin/bash
# partitioned-path GPU tests (host / host-peer ranks on the one GPU)
set -o pipefail
TAG=${1:-dist}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
