#!/bin/bash
# mode 3 against mode 4 on the other BASELINE configs (interleaved)
set -o pipefail
O=gpurun_out/${1:-fdcfg}
mkdir -p $O
for rep in 1 2; do
for mode in 3 4; do
  timeout -k 10 300 python -u tools/configs_bench.py --configs ${2:-p2d_128,p2d_4096,g3_irr,p3d_512} --mode $mode > $O/cfg_m${mode}_$rep.log 2>&1 || { echo "cfg m$mode failed"; tail -20 $O/cfg_m${mode}_$rep.log; exit 1; }
  grep '^{' $O/cfg_m${mode}_$rep.log | python3 -c "import sys,json; [print('m$mode', d['config'], d['it_per_s'], d['ms_per_iter'], d['spmv_variant']) for d in map(json.loads, sys.stdin)]"
done
done
