#!/bin/bash
# Interleaved in-loop bench A/B over environment settings (one per argument
# after the tag; "-" = defaults), two rounds.
#   bash tools/gpu_env_ab.sh TAG - "CGX_SPMV_RESIDENT=0" "CGX_SPMV_GRID=1024"
# (BENCH_ARGS: extra bench.py arguments, e.g. "--workload p3d_512 --steps 40")
set -o pipefail
OUT=gpurun_out/${1:-envab}
shift
mkdir -p $OUT
for r in 1 2; do
  for cfg in "$@"; do
    if [ "$cfg" = "-" ]; then e=""; else e="$cfg"; fi
    env $e timeout -k 10 300 python bench.py --no-cpu --no-general --no-traffic ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
    echo "[$cfg r$r] $(tail -1 $OUT/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["iterations_per_s"], d["config"]["spmv_variant"], r["avg_us"], r["other_kernels_avg_us"])')"
  done
done
