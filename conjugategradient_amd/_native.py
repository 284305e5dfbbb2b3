"""ctypes loader for libcgx.so (the C ABI declared in include/cgx.h).

The library is built in-tree for gfx950 by ``__graft_entry__.build()`` (or
``make -C conjugategradient_amd/csrc``). There is no fallback: if the library
or a gfx950 device is missing, every compute call raises ``CgxError``.

torch, when installed, is imported BEFORE the library is loaded: torch ships
its own libamdhip64 (soname libamdhip64.so.7) and the process must end up with
exactly one HIP runtime, which happens only if torch's copy is loaded first.
"""
from __future__ import annotations

import ctypes as C
import os
import re

try:  # noqa: SIM105 - see module docstring
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libcgx.so")
# (tools/ab_lib.py, the A/B harness, points LIB_PATH at another build and sets
# this to leave entry points an older build lacks unbound)
_AB_BUILD = False
HEADER = os.path.join(os.path.dirname(HERE), "include", "cgx.h")

F64, F32 = 0, 1


class CgxError(RuntimeError):
    """A libcgx call failed (message from cgx_last_error())."""


_lib = None

_vp = C.c_void_p
_i64 = C.c_int64
_i32 = C.c_int
_dbl = C.c_double
_sz = C.c_size_t

# name -> (restype, argtypes)
_SIGS = {
    "cgx_last_error": (C.c_char_p, []),
    "cgx_version": (C.c_char_p, []),
    "cgx_device_count": (_i32, [C.POINTER(_i32)]),
    "cgx_create": (_i32, [_i32, C.POINTER(_vp)]),
    "cgx_destroy": (_i32, [_vp]),
    "cgx_sync": (_i32, [_vp]),
    "cgx_get_stream": (_i32, [_vp, C.POINTER(_vp)]),
    "cgx_get_device": (_i32, [_vp, C.POINTER(_i32)]),
    "cgx_max_work_group_size": (_i32, [_vp, C.POINTER(_i32)]),
    "cgx_alloc": (_i32, [_vp, _sz, C.POINTER(_vp)]),
    "cgx_free": (_i32, [_vp, _vp]),
    "cgx_h2d": (_i32, [_vp, _vp, _vp, _sz]),
    "cgx_h2d_async": (_i32, [_vp, _vp, _vp, _sz]),
    "cgx_d2h": (_i32, [_vp, _vp, _vp, _sz]),
    "cgx_d2d": (_i32, [_vp, _vp, _vp, _sz]),
    "cgx_fill": (_i32, [_vp, _i32, _vp, _dbl, _sz]),
    "cgx_csr_create": (_i32, [_vp, _i64, _i64, _vp, _vp, _vp, _i32, _vp, C.POINTER(_vp)]),
    "cgx_csr_destroy": (_i32, [_vp]),
    "cgx_csr_set_tile": (_i32, [_vp, _i32]),
    "cgx_csr_set_block_order": (_i32, [_vp, _i32]),
    "cgx_csr_block_order_info": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32)]),
    "cgx_csr_variant": (_i32, [_vp, C.POINTER(_i32)]),
    "cgx_csr_set_variant": (_i32, [_vp, _i32]),
    "cgx_csr_set_sell": (_i32, [_vp, _i32]),
    "cgx_csr_split_info": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32)]),
    "cgx_csr_sell_info": (_i32, [_vp, C.POINTER(_i32), C.POINTER(C.c_int64)]),
    "cgx_csr_visit_order": (_i32, [_vp, C.POINTER(_i32)]),
    "cgx_csr_value_codes": (_i32, [_vp, C.POINTER(_i32)]),
    "cgx_csr_templates": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i64)]),
    "cgx_csr_lean_info": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i64), C.POINTER(_i32),
                                 C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32)]),
    "cgx_csr_autotune_record": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32),
                                       C.POINTER(C.c_float), _i32, C.POINTER(_i32)]),
    "cgx_csr_setup_times": (_i32, [_vp, C.POINTER(_dbl), _i32, C.POINTER(_i32)]),
    "cgx_csr_set_lean_team": (_i32, [_vp, _i32]),
    "cgx_csr_lean_team": (_i32, [_vp, C.POINTER(_i32)]),
    "cgx_csr_march_info": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32)]),
    "cgx_csr_stream_bytes": (_i32, [_vp, C.POINTER(C.c_int64)]),
    "cgx_csr_info": (_i32, [_vp, C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64),
                            C.POINTER(_i32)]),
    "cgx_spmv": (_i32, [_vp, _vp, _vp, _vp, _i64]),
    "cgx_dot_acc": (_i32, [_vp, _i32, _i64, _vp, _vp, _vp]),
    "cgx_norm_acc": (_i32, [_vp, _i32, _i64, _vp, _vp]),
    "cgx_sapbx": (_i32, [_vp, _i32, _i64, _vp, _vp, _vp, _vp]),
    "cgx_sambx": (_i32, [_vp, _i32, _i64, _vp, _vp, _vp, _vp]),
    "cgx_saxpby": (_i32, [_vp, _i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "cgx_scalar_div": (_i32, [_vp, _i32, _vp, _vp, _vp]),
    "cgx_cg_create": (_i32, [_vp, _vp, C.POINTER(_vp)]),
    "cgx_cg_destroy": (_i32, [_vp]),
    "cgx_cg_solve": (_i32, [_vp, _vp, _vp, _dbl, _i64, C.POINTER(_i64), C.POINTER(_dbl)]),
    "cgx_cg_begin": (_i32, [_vp, _vp, _vp, _dbl, _i64]),
    "cgx_cg_run": (_i32, [_vp, _i64, C.POINTER(_i64), C.POINTER(_i32)]),
    "cgx_cg_prepare": (_i32, [_vp, _i64]),
    "cgx_cg_rxr": (_i32, [_vp, C.POINTER(_dbl)]),
    "cgx_cg_set_kernel_timing": (_i32, [_vp, _i32]),
    "cgx_cg_kernel_times": (_i32, [_vp, C.POINTER(_dbl), C.POINTER(_i64)]),
    "cgx_cg_kernel_exec_times": (_i32, [_vp, C.POINTER(_dbl), C.POINTER(_i64)]),
    "cgx_cg_config": (_i32, [_vp, _i32, _i32]),
    "cgx_cg_set_mode": (_i32, [_vp, _i32]),
    "cgx_cg_coop_shape": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32),
                                 C.POINTER(_i32)]),
    "cgx_cg_coop_trace": (_i32, [_vp, C.POINTER(C.c_uint64), _i64]),
    "cgx_cg_get_mode": (_i32, [_vp, C.POINTER(_i32)]),
    "cgx_csr_fd_grid": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32)]),
    "cgx_accuracy": (_i32, [_vp, _vp, _vp, _vp, C.POINTER(_dbl)]),
    "cgx_poisson_nnz": (_i64, [_i32, _i32, _i32, _i32, _i64, _i64]),
    "cgx_poisson_fill": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i64, _i64, _vp, _vp, _vp]),
    "cgx_iota": (_i32, [_vp, _i32, _vp, _i64, _dbl]),
    "cgx_nccl_unique_id": (_i32, [C.c_char_p, _sz]),
    "cgx_dist_init": (_i32, [_vp, _i32, _i32, C.c_char_p, _sz]),
    "cgx_dist_init_host": (_i32, [_vp, _i32, _i32, _vp, _vp, _vp, _vp]),
    "cgx_dist_rank": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32)]),
    "cgx_dist_host_async": (_i32, [_vp, _i32]),
    "cgx_csr_halo_async_calls": (_i32, [_vp, C.POINTER(_i64)]),
    "cgx_csr_create_dist": (_i32, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i32,
                                   C.POINTER(_vp)]),
    "cgx_csr_halo_info": (_i32, [_vp, C.POINTER(_i64), C.POINTER(_i32)]),
    "cgx_dist_allreduce_sum": (_i32, [_vp, C.POINTER(_dbl)]),
    "cgx_dist_peer_enable": (_i32, [_vp, C.POINTER(_i32)]),
    "cgx_dist_peer_info": (_i32, [_vp, C.POINTER(_i32)]),
    "cgx_dist_peer_form": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32)]),
    # host-only helpers (no device needed)
    "cgx_plan_ghosts": (_i32, [_i64, _i64, _i64, _vp, _i32, _vp, _vp, C.POINTER(_i64),
                               C.POINTER(C.POINTER(_i64)), _vp]),
    "cgx_plan_remap": (_i32, [_i64, _i64, _i64, _vp, _i64, _vp]),
    "cgx_free_host": (None, [_vp]),
    "cgx_mm_read": (_i32, [C.c_char_p, _i32, C.POINTER(_i64), C.POINTER(_i64),
                           C.POINTER(C.POINTER(_i32)), C.POINTER(C.POINTER(_i32)),
                           C.POINTER(C.POINTER(C.c_double))]),
    "cgx_mm_write_lower": (_i32, [C.c_char_p, _i64, _vp, _vp, _vp, _i32]),
    "cgx_sellp_plan": (_i32, [_vp, _vp, _i64, C.POINTER(_i64), C.POINTER(C.POINTER(_i64)),
                              C.POINTER(_i64), C.POINTER(C.POINTER(_i32)), C.POINTER(_i64),
                              C.POINTER(_i32)]),
    "cgx_sellp_plan_device": (_i32, [_vp, _vp, _vp, _i64, _i64, C.POINTER(_i64),
                                     C.POINTER(C.POINTER(_i64)), C.POINTER(_i64),
                                     C.POINTER(C.POINTER(_i32)), C.POINTER(_i64),
                                     C.POINTER(_i32)]),
    "cgx_sell_plan": (_i32, [_vp, _vp, _i64, _i32, C.POINTER(_i64), C.POINTER(C.POINTER(_i64)),
                             C.POINTER(_i64), C.POINTER(C.POINTER(_i32)), C.POINTER(_i64),
                             C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(_i64)]),
    "cgx_tune_spmv": (_i32, [_vp, _vp, _i32, _vp, _vp, _i32, C.POINTER(_dbl)]),
    "cgx_row_blocks": (_i32, [_vp, _i64, C.POINTER(_i64), C.POINTER(C.POINTER(_i32)),
                              C.POINTER(_i32)]),
}


def lib() -> C.CDLL:
    """Load libcgx.so (once). Raises CgxError if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CgxError(f"{LIB_PATH} not built: run __graft_entry__.build() or "
                           "make -C conjugategradient_amd/csrc")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if _AB_BUILD and not hasattr(L, name):
                continue  # an older A/B build without this entry point
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().cgx_last_error()
        raise CgxError(msg.decode() if msg else f"libcgx error {rc}")


def header_symbols() -> list[str]:
    """Every function name declared in include/cgx.h."""
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(cgx_[a-z0-9_]+)\s*\(", text)))


def device_count() -> int:
    n = _i32(0)
    check(lib().cgx_device_count(C.byref(n)))
    return n.value
