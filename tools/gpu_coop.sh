#!/bin/bash
# Mode 5 (persistent body): GPU tests, then it/s against the auto mode.
set -o pipefail
TAG=${1:-coop}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_coop.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAIL"; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python -u tools/coop_probe.py ${PROBE_ARGS:-} > $OUT/probe.log 2>&1 || { echo "PROBE FAIL"; tail -30 $OUT/probe.log; exit 1; }
grep '^{' $OUT/probe.log
