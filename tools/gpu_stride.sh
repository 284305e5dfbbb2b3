#!/bin/bash
# Plane stride and the 3-D SpMV: the same stencil on grids whose plane is a
# power of two rows (256x256: 512 KB) or not (256x257, 256x255, 257x256);
# time per variant (tune_spmv) and L2 fabric bytes (FETCH_SIZE, one pass per
# grid).
set -o pipefail
TAG=${1:-stride}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
V=${VARIANTS:-10264578,1875970,8194}
G=${GRIDS:-g3:256x256x256,g3:256x257x256,g3:256x255x256,g3:257x256x256}
timeout -k 10 300 python tools/tune_spmv.py --configs $G --variants $V --rounds 4 --iters 10 > $OUT/tune.log 2>&1 || { echo "TUNE FAIL"; tail $OUT/tune.log; exit 1; }
grep '^{' $OUT/tune.log | cut -c1-160
IFS=',' read -ra GL <<< "$G"
for g in "${GL[@]}"; do
  tag=$(echo $g | tr ':x' '__')
  timeout -k 10 -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_$tag -o run --output-format csv -- python3 tools/tune_spmv.py --configs $g --variants $V --rounds 1 --iters 5 > $OUT/pmc_$tag.log 2>&1 || { echo "PMC $g FAIL"; tail $OUT/pmc_$tag.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, os, re
out = "gpurun_out/" + os.environ.get("TAG", "stride")
for d in sorted(glob.glob(out + "/pmc_*/")):
    res = {}
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"k_spmv_dot<double, (\d+)>", r["Kernel_Name"])
            if m:
                res.setdefault(m.group(1), []).append(float(r["Counter_Value"]))
    print(d, {k: round(2 * 1024 * sum(v) / len(v) / 1e9, 4) for k, v in res.items()})
PY
