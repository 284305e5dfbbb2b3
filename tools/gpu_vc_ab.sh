#!/bin/bash
# A/B of the value-code SELL-P SpMV forms (isolated launches, tools/tune_spmv.py)
set -o pipefail
OUT=gpurun_out/${1:-vcab}
mkdir -p $OUT
V=${2:-34818,100354,165890,34834}
timeout -k 10 300 python tools/tune_spmv.py --configs 3d256,2d4096 --variants $V > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
CGX_SPMV_GRID=1280 timeout -k 10 300 python tools/tune_spmv.py --configs 3d256 --variants $V > $OUT/tune_g1280.log 2>&1 || { tail -20 $OUT/tune_g1280.log; exit 1; }
grep config $OUT/tune.log $OUT/tune_g1280.log | cut -c1-170
