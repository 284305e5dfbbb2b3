#!/usr/bin/env python3
"""Write profiles/pmc_spmv_dot.json from the FETCH_SIZE / WRITE_SIZE passes of
tools/gpu_final.sh (gpurun_out/<tag>/pmc_*). FETCH_SIZE is doubled: gfx950
tallies 128-B requests at 64 B (MI355X_MICROARCH.md, HBM/rocprofv3 section).
usage: pmc_to_json.py <tag> [variant]"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 1875970
kern = f"k_spmv_dot<double, {variant}>"


def mean(counter):
    vals = []
    pat = os.path.join(ROOT, "gpurun_out", tag, f"pmc_{counter}", "**", "*counter_collection.csv")
    for f in glob.glob(pat, recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        sys.exit(f"no {counter} samples for {kern}")
    return sum(vals) / len(vals), len(vals)


fetch, nf = mean("FETCH_SIZE")
write, nw = mean("WRITE_SIZE")
n = 256 ** 3
nnz = 7 * n - 6 * 256 ** 2
out = {
    "grid": 256, "n_gpus": 1, "kernel": "k_spmv_dot", "spmv_variant": variant,
    "fetch_size_kb": round(fetch, 1), "write_size_kb": round(write, 1),
    "hbm_bytes_per_launch": int(round((2 * fetch + write) * 1024)),
    "method": ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate runs, of "
               "'python3 bench.py --no-cpu --steps 10 --warmup 2 --profile-steps 0' "
               f"(tools/gpu_final.sh, run {tag}), mean over {nf}/{nw} dispatches of {kern}; "
               "FETCH_SIZE doubled (gfx950 tallies 128-B requests at 64 B, "
               "MI355X_MICROARCH.md HBM/rocprofv3 section); KB = 1024 B"),
    "raw": f"profiles/r02{tag[2:]}_pmc_fetch.txt, profiles/r02{tag[2:]}_pmc_write.txt" if tag.startswith("r2") else f"profiles/{tag}_pmc_spmv.txt",
    "algorithmic_bytes_per_launch": 12 * nnz + 4 * (n + 1) + 16 * n,
    "note": ("SELL-P copy with value codes: per row pair and chunk of 8 slots one 8-byte "
             "word of 4-bit codes into the matrix's value dictionary (2 values at 256^3), "
             "offset patterns per 128-row slice; instead of CSR's 12 B per entry + 4 B rowptr "
             "per row, so traffic is far below the CSR-format algorithmic bytes"
             if variant & 32768 else
             "SELL-P copy: 8 B value per slot (+1.3% padding) and a 1-byte slot mask per row "
             "instead of CSR's 12 B per entry + 4 B rowptr per row, so traffic is below the "
             "CSR-format algorithmic bytes"),
}
json.dump(out, open(os.path.join(ROOT, "profiles", "pmc_spmv_dot.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
