"""Mode 5 (persistent body) against the auto mode on cache-resident problems:
it/s of cgx_cg_run over K bodies (tol 0), after W warmup bodies, per rows-per-
thread choice. One JSON line per (config, mode, R)."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugategradient_amd as cga  # noqa: E402
from conjugategradient_amd._native import check, lib  # noqa: E402
from conjugategradient_amd import workloads  # noqa: E402

CONFIGS = {
    "p2d_128": lambda: ("poisson", (2, 128, 128, 1)),
    "p2d_256": lambda: ("poisson", (2, 256, 256, 1)),
    "p2d_64": lambda: ("poisson", (2, 64, 64, 1)),
    "p2d_180": lambda: ("poisson", (2, 180, 180, 1)),
    "p3d_32": lambda: ("poisson", (3, 32, 32, 32)),
    "p3d_40": lambda: ("poisson", (3, 40, 40, 40)),
    "irr_100k": lambda: ("irr", 100000),
    "irr_400k": lambda: ("irr", 400000),
    "p2d_512": lambda: ("poisson", (2, 512, 512, 1)),
    "p2d_1024": lambda: ("poisson", (2, 1024, 1024, 1)),
    "p3d_100": lambda: ("poisson", (3, 100, 100, 100)),
    "p3d_164k": lambda: ("poisson", (3, 64, 64, 40)),
    "p3d_80": lambda: ("poisson", (3, 80, 80, 80)),
    "p2d_700": lambda: ("poisson", (2, 700, 700, 1)),
    "irr_200k": lambda: ("irr", 200000),
    "p3d_60": lambda: ("poisson", (3, 60, 60, 60)),
    "p2d_400": lambda: ("poisson", (2, 400, 400, 1)),
    "g3": lambda: ("g3", None),
}


VARIANTS = [(0, None, None, None), (5, "1", "0", "1024"), (5, "1", "0", "512"), (5, "1", "1", "512")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="p2d_128,p3d_40,irr_100k")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="", help="R:form:threads,... (mode 5 shapes to time; "
                    "form 0 write-through, 1 tagged, 2 streamed; R 0: the fewest that fit)")
    ap.add_argument("--base-env", default="", help="K=V,... for the mode-0 runs (e.g. "
                    "CGX_COOP_STREAM=0: the auto mode without the streamed form)")
    a = ap.parse_args()
    base_env = dict(kv.split("=", 1) for kv in a.base_env.split(",") if kv)
    global VARIANTS
    if a.shapes:
        VARIANTS = [(0, None, None, None)] + [(5, *sh.split(":")) for sh in a.shapes.split(",")]
    L = lib()
    q = cga.Queue(0)
    import torch
    for name in a.configs.split(","):
        kind, arg = CONFIGS[name]()
        if kind == "poisson":
            m = cga.Matrix.poisson(q, *arg)
        elif kind == "g3":
            rp, cl, vl = workloads.host_csr("g3_standin")
            m = cga.Matrix(q, vl, cl, rp)
        else:
            rp, cl, vl = workloads.irregular_spd(arg)
            m = cga.Matrix(q, vl, cl, rp)
        n = m.N()
        A = m.schedule()
        b = torch.arange(1, n + 1, dtype=torch.float64, device="cuda")
        res = {}
        for rnd in range(a.rounds):
            for mode, R, tg, nt in VARIANTS:
                for k, v in base_env.items():
                    if R:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
                if R:
                    if R != "0":
                        os.environ["CGX_COOP_R"] = R
                    os.environ["CGX_COOP_TAGR"] = "1" if tg == "1" else "0"
                    os.environ["CGX_COOP_STREAM"] = "1" if tg == "2" else "0"
                    os.environ["CGX_COOP_NT"] = nt
                x = torch.zeros(n, dtype=torch.float64, device="cuda")
                torch.cuda.synchronize()
                cg = C.c_void_p()
                check(L.cgx_cg_create(q.handle, A, C.byref(cg)))
                if L.cgx_cg_set_mode(cg, mode) != 0:
                    L.cgx_cg_destroy(cg)
                    continue
                me = C.c_int()
                check(L.cgx_cg_get_mode(cg, C.byref(me)))
                check(L.cgx_cg_begin(cg, C.c_void_p(b.data_ptr()), C.c_void_p(x.data_ptr()), 0.0,
                                     a.warmup + a.steps))
                bodies, stopped = C.c_int64(), C.c_int()
                check(L.cgx_cg_run(cg, a.warmup, C.byref(bodies), C.byref(stopped)))
                check(L.cgx_cg_prepare(cg, a.steps))
                q.wait()
                t0 = time.perf_counter()
                check(L.cgx_cg_run(cg, a.steps, C.byref(bodies), C.byref(stopped)))
                q.wait()
                dt = time.perf_counter() - t0
                rxr = C.c_double()
                check(L.cgx_cg_rxr(cg, C.byref(rxr)))
                check(L.cgx_cg_destroy(cg))
                key = (mode if mode != 5 else f"5/R{R}/form{tg}/nt{nt}")
                ran = bodies.value - a.warmup
                res.setdefault(key, []).append((dt / max(ran, 1) * 1e6, ran, me.value, rxr.value))
                os.environ.pop("CGX_COOP_R", None)
                os.environ.pop("CGX_COOP_TAGR", None)
                os.environ.pop("CGX_COOP_NT", None)
                os.environ.pop("CGX_COOP_STREAM", None)
        for k, v in res.items():
            us = sorted(t[0] for t in v)
            print(json.dumps({"config": name, "n": n, "mode": k, "mode_eff": v[0][2], "bodies": v[0][1],
                              "us_per_body_min": round(us[0], 3), "us_per_body_med": round(us[len(us) // 2], 3),
                              "it_per_s": round(1e6 / us[0], 1), "rxr": v[0][3]}), flush=True)


if __name__ == "__main__":
    main()
