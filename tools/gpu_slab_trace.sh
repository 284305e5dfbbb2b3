#!/bin/bash
# kernel trace of the 256x256x32 slab body (graph replay): per-kernel
# durations and the gaps between consecutive kernels
set -o pipefail
OUT=gpurun_out/${1:-slabtr}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 tools/slab_bench.py 3,256,256,32,400 > $OUT/run.log 2>&1 || { echo TRACE_FAIL; tail $OUT/run.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, statistics as S
out = sys.argv[1]
f = glob.glob(out + "/tr/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# the last 200 kernels of the run (steady state)
rows = [r for r in rows if "k_" in r["Kernel_Name"]][-300:]
dur, gap = {}, {}
for a, b in zip(rows, rows[1:]):
    na = a["Kernel_Name"].split("(")[0].replace("void cgx::", "").replace("(anonymous namespace)::", "")
    nb = b["Kernel_Name"].split("(")[0].replace("void cgx::", "").replace("(anonymous namespace)::", "")
    dur.setdefault(na, []).append((int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3)
    gap.setdefault(na + " -> " + nb, []).append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
for k, v in dur.items():
    print(f"dur {k}: median {S.median(v):.2f} us (n={len(v)})")
for k, v in gap.items():
    print(f"gap {k}: median {S.median(v):.2f} us (n={len(v)})")
PY
