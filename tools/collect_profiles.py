#!/usr/bin/env python3
"""Copy a tools/gpu_record.sh run's summaries from gpurun_out/<tag>/ into
profiles/<prefix>_* (tracked): the GPU test log, smoke, the driver-command
bench line, the rocprofv3 --kernel-trace --stats summary of that command,
per-kernel HBM bytes from its FETCH_SIZE / WRITE_SIZE PMC passes, and the
per-config lines.

    python tools/collect_profiles.py r3b r03b
"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

tag, prefix = sys.argv[1], sys.argv[2]
src = os.path.join(ROOT, "gpurun_out", tag)
dst = os.path.join(ROOT, "profiles")
for name, out in (("pytest_gpu.log", "pytest_gpu.log"), ("smoke.log", "smoke.log"),
                  ("bench_driver.log", "bench_driver.log"), ("configs.log", "configs.log"),
                  ("prof/bench_kernel_stats.csv", "bench_kernel_stats.csv")):
    p = os.path.join(src, name)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, f"{prefix}_{out}"))
        print("copied", name)
sums: dict = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(src, f"pmc_{ctr}", "**", "*counter_collection.csv"),
                       recursive=True):
        bench.pmc_accumulate(open(f), ctr, sums)
if sums:
    out = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate runs of "
                     "'python3 bench.py --no-cpu --no-general --steps 10 --warmup 2 "
                     "--profile-steps 0' (tools/gpu_record.sh); per dispatch (2 x FETCH_SIZE + "
                     "WRITE_SIZE) x 1024 B (gfx950 FETCH correction, MI355X_MICROARCH.md)",
           "run": tag,
           "dispatches": {k: {c: v[1] for c, v in d.items()} for k, d in sums.items()},
           "hbm_bytes_per_dispatch": bench.pmc_bytes(sums)}
    json.dump(out, open(os.path.join(dst, f"{prefix}_pmc_bytes.json"), "w"), indent=1)
    print("wrote", f"{prefix}_pmc_bytes.json")
