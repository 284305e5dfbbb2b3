#!/usr/bin/env python3
"""bench.py on every SURVEY §8(d) configuration, one GPU, one child process
each (bench.py --workload W), so every config gets the headline line's
fields: `value` on the compulsory bytes of the streamed formats,
`iteration_frac`, the dominant kernel's `roofline` (HIP-event time, `frac`,
and `traffic` from rocprofv3 PMC passes of that same shape, variant and
mode), and `csr_equivalent_GBs`.

  p2d_128     128^2 Poisson read from tests/golden/poisson2d_128.mtx
  p2d_4096    4096^2 Poisson (device generator)
  p3d_256     256^3 Poisson (the headline workload)
  p3d_512     512^3 Poisson on one GPU (the 8-GPU strong-scaling problem)
  g3_standin  the G3_circuit stand-in: seeded irregular SPD, N = 1,585,478

    python tools/configs_bench.py [--configs p2d_128,...] [--no-traffic]

Prints one JSON line per config (bench.py's line) and a summary table.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (steps, warmup, profile steps): a few hundred ms of timed bodies each
PLAN = {"p2d_128": (600, 20, 200), "p2d_4096": (400, 20, 100), "p3d_256": (400, 20, 100),
        "p3d_512": (80, 5, 20), "g3_standin": (2000, 50, 200)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="p2d_128,p2d_4096,p3d_256,p3d_512,g3_standin")
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--no-traffic", action="store_true")
    a = ap.parse_args()
    rows = []
    for name in a.configs.split(","):
        steps, warm, prof = PLAN[name]
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", name,
               "--steps", str(steps), "--warmup", str(warm), "--profile-steps", str(prof),
               "--no-cpu", "--no-general", "--mode", str(a.mode)]
        if a.no_traffic:
            cmd.append("--no-traffic")
        p = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, timeout=900)
        if p.returncode != 0:
            print(json.dumps({"config": name, "error": p.stderr[-2000:]}), flush=True)
            continue
        line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
        line["config"]["name"] = name
        print(json.dumps(line), flush=True)
        rows.append((name, line))
    print("\n| config | it/s | GB/s (compulsory) | iteration_frac | dominant kernel | "
          "avg us | frac | traffic / compulsory | CSR-equivalent GB/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name, ln in rows:
        r = ln.get("roofline") or {}
        kern = (f"{r.get('kernel')}{r['template']} (whole body)" if r.get("template")
                else f"{r.get('kernel')}<{ln['config']['spmv_variant']}>")
        us = r.get("us_per_body") or r.get("avg_us")
        print(f"| {name} | {ln['iterations_per_s']:,} | {ln['achieved_GBs']:,} | {ln['iteration_frac']} | "
              f"{kern} | {us} | "
              f"{r.get('frac')} | {r.get('traffic_ratio_to_compulsory')} | "
              f"{ln['csr_equivalent_GBs']:,} |", flush=True)


if __name__ == "__main__":
    main()
