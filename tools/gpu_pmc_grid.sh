#!/bin/bash
# 3-D SpMV (templates) at several grid caps: time (tune_spmv) and L2 fabric
# traffic (rocprofv3 --pmc FETCH_SIZE, then TCC_HIT_sum / TCC_MISS_sum, one
# group per run). Also 256^3 mode 4 against mode 3 in the loop.
set -o pipefail
TAG=${1:-pmcg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
V=10264578
for g in 2048 1024 768 512; do
  CGX_SPMV_GRID=$g timeout -k 10 200 python tools/tune_spmv.py --configs 3d256 --variants $V --rounds 3 --iters 10 > $OUT/tune_g$g.log 2>&1 || { echo "TUNE $g FAIL"; tail $OUT/tune_g$g.log; exit 1; }
  grep '^{' $OUT/tune_g$g.log | cut -c1-120
  for C in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    n=$(echo $C | cut -d' ' -f1)
    CGX_SPMV_GRID=$g timeout -k 10 -s KILL 200 rocprofv3 --pmc $C -d $OUT/pmc_g${g}_$n -o run --output-format csv -- python3 tools/tune_spmv.py --configs 3d256 --variants $V --rounds 1 --iters 5 > $OUT/pmc_g${g}_$n.log 2>&1 || { echo "PMC $g $n FAIL"; tail $OUT/pmc_g${g}_$n.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, os
out = "gpurun_out/" + os.environ.get("TAG", "pmcg")
for g in (2048, 1024, 768, 512):
    res = {}
    for n in ("FETCH_SIZE", "TCC_HIT_sum"):
        for f in glob.glob(f"{out}/pmc_g{g}_{n}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_spmv_dot<double, 10264578>" in r["Kernel_Name"]:
                    res.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    s = {k: sum(v) / len(v) for k, v in res.items()}
    fb = 2 * s.get("FETCH_SIZE", 0) * 1024
    h, m = s.get("TCC_HIT_sum", 0), s.get("TCC_MISS_sum", 0)
    print(f"grid {g}: fetch {fb/1e9:.4f} GB (x2 corrected), L2 hit {h/(h+m+1e-9):.3f}, n={len(res.get('FETCH_SIZE', []))}")
PY
for m in 3 4 3 4; do
  timeout -k 10 300 python bench.py --mode $m --steps 200 --warmup 10 --no-cpu --no-general --no-traffic > $OUT/bench_m$m.log 2>&1 || { echo "BENCH m$m FAIL"; tail $OUT/bench_m$m.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_m$m.log') if l.startswith('{')][-1]); r=d['roofline']; print('mode $m', d['iterations_per_s'], r['kernel'], r['avg_us'], r['other_kernels_avg_us'])"
done
