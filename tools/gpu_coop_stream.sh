#!/bin/bash
# Mode 5's streamed form: the coop GPU tests, then it/s of the auto mode
# without it (CGX_COOP_STREAM=0) against it on problems past the register
# forms.
set -o pipefail
OUT=gpurun_out/${1:-coopst}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_coop.py -x -v -s --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
grep -E "passed|failed|g3 streamed" $OUT/pytest.log | tail -5
timeout -k 10 500 python -u tools/coop_probe.py --configs ${CONFIGS:-g3,irr_400k,irr_200k,irr_100k,p2d_512,p2d_700,p2d_1024,p3d_164k,p3d_80,p3d_100} --steps ${STEPS:-500} --warmup 50 --rounds 2 --shapes ${SHAPES:-0:2:1024} --base-env CGX_COOP_STREAM=0 > $OUT/probe.log 2>&1 || { tail -30 $OUT/probe.log; exit 1; }
cat $OUT/probe.log | grep config
