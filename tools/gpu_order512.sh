#!/bin/bash
# A/B: the slice visit order ($CGX_SELL_ORDER=1, cgx_abi.cpp sell_visit_order)
# at 512^3 on one GPU, where p (1.07 GB) does not fit the Infinity Cache and
# the +-D gathers are 2 MB apart. Interleaved runs of the bench line.
#   tools/gpu_order512.sh TAG
set -o pipefail
TAG=${1:-order512}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for ord in 0 1; do
    CGX_SELL_ORDER=$ord timeout -k 10 240 python3 bench.py --workload p3d_512 --steps 80 \
        --warmup 5 --profile-steps 20 --no-cpu --no-general --no-traffic \
        > $OUT/o${ord}_$rep.log 2>&1 || { echo "FAIL order=$ord rep=$rep"; tail -20 $OUT/o${ord}_$rep.log; exit 1; }
    python3 - "$OUT/o${ord}_$rep.log" "$ord" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"order={sys.argv[2]} it/s={d['iterations_per_s']} variant={d['config']['spmv_variant']} "
      f"spmv_us={r['avg_us']} others={r['other_kernels_avg_us']}", flush=True)
EOF
  done
done
