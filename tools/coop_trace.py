"""Phase stamps of the persistent body (mode 5, $CGX_COOP_TRACE): for bodies
8-15 of a launch, per workgroup, the wall clock (100 MHz) at body start (0),
SpMV done (1), p.Ap partial ready (2), p.Ap exchanged (3), r.r partial
ready (4), next gathers done (5), r.r exchanged (6). Prints medians of each
phase's length and of the exchanges' skew and latency past the last
arrival, in microseconds."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["CGX_COOP_TRACE"] = "1"
import conjugategradient_amd as cga  # noqa: E402
from conjugategradient_amd._native import check, lib  # noqa: E402


VARIANTS = ["0", "1"]  # $CGX_COOP_STREAM: the register form, the streamed form


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="64,128,180")
    a = ap.parse_args()
    L = lib()
    q = cga.Queue(0)
    import torch
    for nx in [int(v) for v in a.grids.split(",")]:
        m = cga.Matrix.poisson(q, 2, nx, nx, 1)
        n = m.N()
        A = m.schedule()
        b = torch.arange(1, n + 1, dtype=torch.float64, device="cuda")
        for v in VARIANTS:
            os.environ["CGX_COOP_STREAM"] = v
            x = torch.zeros(n, dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            cg = C.c_void_p()
            check(L.cgx_cg_create(q.handle, A, C.byref(cg)))
            if L.cgx_cg_set_mode(cg, 5) != 0:
                check(L.cgx_cg_destroy(cg))
                continue
            check(L.cgx_cg_config(cg, 8, 0))  # 64 bodies per launch
            R, NT, G, T = C.c_int(), C.c_int(), C.c_int(), C.c_int()
            check(L.cgx_cg_coop_shape(cg, C.byref(R), C.byref(NT), C.byref(G), C.byref(T)))
            check(L.cgx_cg_begin(cg, C.c_void_p(b.data_ptr()), C.c_void_p(x.data_ptr()), 0.0, 64))
            bodies, stopped = C.c_int64(), C.c_int()
            check(L.cgx_cg_run(cg, 64, C.byref(bodies), C.byref(stopped)))
            buf = (C.c_uint64 * (128 * 64))()
            check(L.cgx_cg_coop_trace(cg, buf, 128 * 64))
            check(L.cgx_cg_destroy(cg))
            t = np.frombuffer(buf, dtype=np.uint64).reshape(128, 8, 8)[:G.value].astype(np.float64) / 100.0
            ph = np.diff(t[:, :, :7], axis=2)  # [wg][body][phase step]
            med = np.median(ph.reshape(-1, 6), axis=0)
            # exchange A: last arrival (max of phase 2) -> each WG's collect (3)
            lastA = t[:, :, 2].max(axis=0)
            latA = np.median(t[:, :, 3] - lastA[None, :])
            skewA = np.median(t[:, :, 2].max(axis=0) - t[:, :, 2].min(axis=0))
            lastB = t[:, :, 4].max(axis=0)
            latB = np.median(t[:, :, 6] - lastB[None, :])
            skewB = np.median(t[:, :, 4].max(axis=0) - t[:, :, 4].min(axis=0))
            body = np.median(np.diff(t[0, :, 0]))
            print(f"p2d_{nx} n={n} R={R.value} G={G.value} NT={v[1]} nap={v[2]} tagged={T.value} "
                  f"body {body:.2f} us | "
                  f"spmv {med[0]:.2f} sumA {med[1]:.2f} xA {med[2]:.2f} upd+sumB {med[3]:.2f} "
                  f"gath {med[4]:.2f} xB {med[5]:.2f} | skewA {skewA:.2f} latA {latA:.2f} "
                  f"skewB {skewB:.2f} latB {latB:.2f}", flush=True)


if __name__ == "__main__":
    main()
