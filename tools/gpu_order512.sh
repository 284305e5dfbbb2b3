#!/bin/bash
# A/B: the slice visit order ($CGX_SELL_ORDER=1, cgx_abi.cpp sell_visit_order;
# $CGX_SELL_ORDER_CHUNK slices of a plane per chunk) at 512^3 on one GPU,
# where p (1.07 GB) does not fit the Infinity Cache and the +-D gathers are
# 2 MB apart. Interleaved runs of the bench line. Arguments after TAG: the
# order settings to compare ("0" = natural order, else a chunk size).
#   tools/gpu_order512.sh TAG [WORKLOAD] [SETTINGS...]
set -o pipefail
TAG=${1:-order512}
WL=${2:-p3d_512}
shift 2
SETS=${@:-0 128}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for c in $SETS; do
    # auto: no setting (the library's own choice); 0: natural order; N: chunks of N
    if [ "$c" = auto ]; then unset CGX_SELL_ORDER CGX_SELL_ORDER_CHUNK
    elif [ "$c" = 0 ]; then export CGX_SELL_ORDER=0; unset CGX_SELL_ORDER_CHUNK
    else export CGX_SELL_ORDER=1 CGX_SELL_ORDER_CHUNK=$c; fi
    timeout -k 10 240 python3 bench.py --workload $WL \
        --steps 80 --warmup 5 --profile-steps 20 --no-cpu --no-general --no-traffic \
        > $OUT/c${c}_$rep.log 2>&1 || { echo "FAIL chunk=$c rep=$rep"; tail -20 $OUT/c${c}_$rep.log; exit 1; }
    python3 - "$OUT/c${c}_$rep.log" "$c" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"chunk={sys.argv[2]} it/s={d['iterations_per_s']} variant={d['config']['spmv_variant']} "
      f"spmv_us={r['avg_us']} others={r['other_kernels_avg_us']}", flush=True)
EOF
  done
done
