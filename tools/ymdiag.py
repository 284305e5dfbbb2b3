import ctypes as C, os, sys, numpy as np
sys.path.insert(0, "/root/repo")
import conjugategradient_amd as cga
from conjugategradient_amd._native import check, lib
L = lib(); q = cga.Queue(0)
for dims in [(3, 256, 256, 32)]:
    try:
        m = cga.Matrix.poisson(q, *dims); m.schedule()
    except Exception as e:
        print("create with autotune failed:", e, flush=True)
    os.environ["CGX_SPMV_VARIANT"] = "10264578"
    m = cga.Matrix.poisson(q, *dims)
    v0 = C.c_int(); check(L.cgx_csr_variant(m.schedule(), C.byref(v0)))
    st, off, run = C.c_int(), C.c_int(), C.c_int()
    check(L.cgx_csr_march_info(m.schedule(), C.byref(st), C.byref(off), C.byref(run)))
    print(dims, "variant", v0.value, "march", st.value, off.value, run.value, flush=True)
    x = np.random.default_rng(0).standard_normal(m.N())
    ref = None
    for v in [10264578, 12361730, 29138946, 20750338, 20750336]:
        rc = L.cgx_csr_set_variant(m.schedule(), v)
        if rc:
            print(v, "set_variant rc", rc, L.cgx_last_error().decode(), flush=True); continue
        got = C.c_int(); check(L.cgx_csr_variant(m.schedule(), C.byref(got)))
        y = cga.Vector(q, m.N())
        try:
            cga.VectorOperations(q).spmv(m, cga.Vector(q, x), y, m.NNZ(), count=m.N())
            yy = y.to_numpy()
            if ref is None: ref = yy
            print(v, "->", got.value, "bitexact", bool(np.array_equal(yy, ref)), flush=True)
        except Exception as e:
            print(v, "->", got.value, "ERROR", e, flush=True)
