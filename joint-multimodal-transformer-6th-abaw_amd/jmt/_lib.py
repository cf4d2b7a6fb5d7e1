"""ctypes binding of libjmt_hip.so (include/jmt.h).

The library is built in-tree by csrc/Makefile (`python -m jmt.build` or __graft_entry__.build()).
There is NO fallback: if the library is missing or a call fails, this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# JMT_LIB selects another build of the same ABI (csrc `make bounds`: build/bounds/libjmt_hip.so
# with device-side index checks); default: the in-tree library
LIB_PATH = os.environ.get("JMT_LIB") or os.path.join(_HERE, "libjmt_hip.so")

F32, BF16, F16 = 0, 1, 2
OK, ERR_ARG, ERR_HIP, ERR_UNSUPPORTED = 0, -1, -2, -3     # include/jmt.h

c_i64 = C.c_int64
c_vp = C.c_void_p
c_int = C.c_int
c_f = C.c_float
c_fp = C.POINTER(C.c_float)


class GemmDesc(C.Structure):
    _fields_ = [
        ("ab_dtype", c_int), ("c_dtype", c_int), ("aux_dtype", c_int),
        ("M", c_int), ("N", c_int), ("K", c_int),
        ("a", c_vp * 8), ("b", c_vp * 8), ("c", c_vp * 8),
        ("n_a", c_int), ("n_b", c_int), ("n_c", c_int),
        ("a_mode", c_int), ("b_mode", c_int), ("c_mode", c_int),
        ("a_kseg", c_int), ("b_kseg", c_int),
        ("a_kmajor", c_int), ("b_kmajor", c_int),
        ("lda", c_i64), ("ldb", c_i64), ("ldc", c_i64), ("ldaux", c_i64),
        ("batch0", c_int), ("batch1", c_int),
        ("sA0", c_i64), ("sA1", c_i64), ("sB0", c_i64), ("sB1", c_i64),
        ("sC0", c_i64), ("sC1", c_i64),
        ("alpha", c_f), ("beta", c_f),
        ("bias", c_vp), ("bias_mode", c_int), ("relu", c_int),
        ("aux", c_vp),
        ("splits", c_int),
        ("workspace", c_vp), ("ws_bytes", C.c_size_t),
        ("bias_tab", c_vp * 8), ("n_bias", c_int),
        ("dbias_tab", c_vp * 8), ("n_dbias", c_int), ("dbias_acc", c_int),
        ("dbias_ws", c_vp), ("dbias_ws_bytes", C.c_size_t),
    ]


# name -> (restype, argtypes)
_PROTOS = {
    "jmt_abi_version": (c_int, []),
    "jmt_last_error": (C.c_char_p, []),
    "jmt_kernel_count": (c_int, []),
    "jmt_bounds_violations": (C.c_longlong, [c_int]),
    "jmt_gemm": (c_int, [C.POINTER(GemmDesc), c_vp]),
    "jmt_gemm_workspace_bytes": (C.c_size_t, [c_int, c_int, c_int, c_int]),
    "jmt_gemm_plan_splits": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "jmt_gemm_set_debug": (None, [c_int]),
    "jmt_gemm_trace_read": (c_int, [c_vp, c_int]),
    "jmt_l2norm_fwd": (c_int, [c_int, c_int, c_i64, c_int, c_vp, c_i64, c_vp, c_i64, c_vp, c_f,
                               c_vp]),
    "jmt_l2norm_bwd": (c_int, [c_int, c_int, c_int, c_i64, c_int, c_vp, c_i64, c_vp, c_i64, c_vp,
                               c_f, c_vp, c_i64, c_vp]),
    "jmt_layernorm_fwd": (c_int, [c_int, c_int, c_i64, c_int, c_vp, c_i64, c_vp, c_i64, c_vp,
                                  c_vp, c_f, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "jmt_layernorm_bwd_blocks": (c_int, [c_i64]),
    "jmt_layernorm_bwd": (c_int, [c_int, c_int, c_int, c_i64, c_int, c_vp, c_i64, c_vp, c_i64,
                                  c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_int,
                                  c_vp, c_vp]),
    "jmt_layernorm_bwd_dsum": (c_int, [c_int, c_int, c_int, c_i64, c_int, c_vp, c_i64, c_vp,
                                       c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp,
                                       c_vp, c_vp, c_int, c_vp, c_vp]),
    "jmt_layernorm_fwd_grouped": (c_int, [c_int, c_int, c_int, c_i64, c_int, c_vp, c_i64, c_i64,
                                          c_vp, c_i64, c_i64, c_vp, c_vp, c_f, c_vp, c_i64, c_i64,
                                          c_vp, c_vp, c_vp]),
    "jmt_layernorm_bwd_grouped": (c_int, [c_int, c_int, c_int, c_int, c_i64, c_int, c_vp, c_i64,
                                          c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp,
                                          c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_int,
                                          c_vp, c_vp]),
    "jmt_softmax_fwd": (c_int, [c_int, c_i64, c_int, c_vp, c_i64, c_f, c_vp, c_i64, c_vp]),
    "jmt_softmax_bwd": (c_int, [c_int, c_int, c_i64, c_int, c_vp, c_i64, c_vp, c_i64, c_f, c_vp,
                                c_i64, c_vp]),
    "jmt_attn_supported": (c_int, [c_int, c_int]),
    "jmt_attn_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_i64, c_i64, c_vp,
                             c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_f, c_vp,
                             c_vp]),
    "jmt_attn_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_i64, c_i64, c_vp,
                             c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64,
                             c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_f, c_vp]),
    "jmt_attn_short_supported": (c_int, [c_int, c_int, c_int, c_int]),
    "jmt_attn_short_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_i64, c_i64,
                                   c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                                   c_f, c_vp, c_vp]),
    "jmt_attn_short_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_i64, c_i64,
                                   c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                                   c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64,
                                   c_i64, c_vp, c_i64, c_i64, c_f, c_vp]),
    "jmt_attn_dkdv": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_i64, c_vp,
                              c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64,
                              c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp]),
    "jmt_noop": (c_int, [c_vp]),
    "jmt_small_attn_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_i64, c_i64,
                                   c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                                   c_f, c_vp, c_vp]),
    "jmt_small_attn_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_i64, c_i64,
                                   c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                                   c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64,
                                   c_i64, c_f, c_vp]),
    "jmt_colsum_blocks": (c_int, [c_i64]),
    "jmt_layernorm_bwd_grouped_blocks": (c_int, [c_i64]),
    "jmt_colsum": (c_int, [c_int, c_i64, c_int, c_vp, c_i64, c_vp, c_int, c_vp, c_vp]),
    "jmt_colsum_grouped": (c_int, [c_int, c_int, c_i64, c_int, c_vp, c_i64, c_i64, c_vp, c_int,
                                   c_vp, c_vp]),
    "jmt_copy2d": (c_int, [c_int, c_int, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                           c_int, c_vp]),
    "jmt_ccc_stats": (c_int, [c_int, c_int, c_i64, c_int, c_vp, c_vp, c_f, c_f, c_f, c_vp, c_vp]),
    "jmt_ccc_finish": (c_int, [c_int, c_int, c_vp, c_i64, c_f, c_vp, c_vp, c_vp]),
    "jmt_ccc_finish_add": (c_int, [c_int, c_int, c_vp, c_i64, c_f, c_vp, c_vp, c_vp, c_vp]),
    "jmt_ccc_bwd": (c_int, [c_int, c_int, c_i64, c_int, c_vp, c_vp, c_f, c_f, c_f, c_vp, c_vp,
                            c_vp, c_vp]),
    "jmt_mask_indices": (c_int, [c_i64, c_vp, c_f, c_vp, c_vp, c_vp]),
    "jmt_vp_scatter": (c_int, [c_i64] + [c_vp] * 9 + [c_f, c_i64] + [c_vp] * 6),
    "jmt_vp_smooth": (c_int, [c_i64, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "jmt_head_fwd": (c_int, [c_int, c_int, c_i64, c_int, c_int, c_vp, c_i64, c_vp, c_vp, c_vp,
                             c_vp, c_vp, c_vp, c_i64, c_vp]),
    "jmt_head_bwd": (c_int, [c_int, c_int, c_i64, c_int, c_int, c_vp, c_i64, c_vp, c_vp, c_vp,
                             c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "jmt_head_bwd_workspace_bytes": (C.c_size_t, [c_i64]),
    "jmt_ce_stats": (c_int, [c_int, c_i64, c_int, c_vp, c_vp, c_f, c_f, c_vp, c_vp, c_vp]),
    "jmt_ce_finish": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp]),
    "jmt_ce_bwd": (c_int, [c_int, c_i64, c_int, c_vp, c_vp, c_f, c_f, c_vp, c_vp, c_vp, c_vp,
                           c_vp]),
    "jmt_ce_labels": (c_int, [c_i64, c_int, c_vp, c_f, c_f, c_vp, c_vp]),
    "jmt_vp_ccc": (c_int, [c_i64] + [c_vp] * 6),
    "jmt_amp_check": (c_int, [c_i64, c_vp, c_vp, c_vp]),
    "jmt_sgd_step_amp": (c_int, [c_i64, c_vp, c_vp, c_vp, c_f, c_f, c_f, c_f, c_int, c_int, c_vp,
                                 c_vp, c_int, c_vp]),
    "jmt_sgd_step_amp_zero": (c_int, [c_i64, c_vp, c_vp, c_vp, c_f, c_f, c_f, c_f, c_int, c_int,
                                      c_vp, c_vp, c_int, c_vp]),
    "jmt_amp_update": (c_int, [c_vp, c_f, c_f, c_int, c_vp]),
    "jmt_gather_rows": (c_int, [c_int, c_int, c_i64, c_int, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64,
                                c_vp]),
    "jmt_sgd_step": (c_int, [c_i64, c_vp, c_vp, c_vp, c_f, c_f, c_f, c_f, c_int, c_int, c_f,
                             c_vp, c_int, c_vp]),
    "jmt_sgd_step_zero": (c_int, [c_i64, c_vp, c_vp, c_vp, c_f, c_f, c_f, c_f, c_int, c_int, c_f,
                                  c_vp, c_int, c_vp]),
}

EXPORTED = tuple(_PROTOS)

_lib = None


class JMTError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load (once) and return the library handle.  Raises if it is missing: no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise JMTError(f"libjmt_hip.so not found at {path}: build it with "
                       f"`make -C joint-multimodal-transformer-6th-abaw_amd/csrc` "
                       f"(or __graft_entry__.build()); there is no CPU/torch fallback")
    lib = C.CDLL(path)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.jmt_abi_version() != 7:
        raise JMTError("libjmt_hip.so ABI version mismatch")
    cfg = int(os.environ.get("JMT_GEMM_CFG", "0"))   # development: force a GEMM pipeline config
    dbg = int(os.environ.get("JMT_GEMM_DBG", "0"))   # development: gemm.hip ablation flags
    if cfg or dbg:
        lib.jmt_gemm_set_debug((cfg << 8) | (dbg & 0xff))
    _lib = lib
    return lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = load().jmt_last_error().decode(errors="replace")
        raise JMTError(f"{what or 'jmt'} failed ({rc}): {msg}")


def call(name: str, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    check(rc, name)
    return rc
