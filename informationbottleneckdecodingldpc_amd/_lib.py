"""ctypes binding of libibldpc.so (include/ibldpc.h).

There is no CPU fallback: if the library is missing or no GPU is visible, decode calls
raise. ``load()`` can be used on a CPU-only machine (the library links against the HIP
runtime, which loads without a device) to inspect symbols or call the host-only
``ibl_map_node_connections``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# IBLDPC_LIB selects an alternative in-tree build (kernel variants, see tools/variants.py)
LIB_PATH = os.environ.get("IBLDPC_LIB") or os.path.join(_HERE, "libibldpc.so")

IBL_OK, IBL_EINVAL, IBL_EHIP, IBL_ENOMEM, IBL_EUNSUPPORTED = 0, -1, -2, -3, -4
IBL_U8, IBL_I32, IBL_F32, IBL_F64 = 1, 2, 3, 4
IBL_MINSUM, IBL_BP = 0, 1
IBL_FLAG_FORCE_GENERIC = 1
IBL_PATH_AUTO, IBL_PATH_PASSES, IBL_PATH_FUSED = 0, 1, 2

# every symbol declared in include/ibldpc.h
EXPORTS = [
    "ibl_version", "ibl_last_error", "ibl_device_count", "ibl_map_node_connections",
    "ibl_graph_create", "ibl_graph_info", "ibl_graph_destroy",
    "ibl_ib_create", "ibl_ib_path", "ibl_ib_set_path", "ibl_ib_path_in_use", "ibl_ib_fused_ncw", "ibl_ib_decode",
    "ibl_ib_set_small_batch", "ibl_ib_small_batch",
    "ibl_ib_destroy",
    "ibl_float_create", "ibl_float_decode", "ibl_float_destroy", "ibl_count_below",
    "ibl_float_set_path", "ibl_float_path_in_use", "ibl_float_folded", "ibl_float_input_check",
    "ibl_float_set_small_batch", "ibl_float_small_batch",
    "ibl_ib_timing", "ibl_ib_timing_read", "ibl_float_timing", "ibl_float_timing_read",
    "ibl_channel_sample",
    "ibl_encoder_create",
    "ibl_encoder_algorithm",
    "ibl_encode",
    "ibl_encoder_destroy",
    "ibl_random_bits",
    "ibl_count_errors",
    "ibl_shard_range", "ibl_comm_unique_id", "ibl_comm_create", "ibl_comm_broadcast", "ibl_comm_allreduce_sum_i64",
    "ibl_comm_destroy",
]
IBL_COMM_ID_BYTES = 128


class IBLError(RuntimeError):
    pass


_lib = None
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_vp = ctypes.c_void_p
_i32, _i64 = ctypes.c_int32, ctypes.c_int64


def load():
    """Load libibldpc.so (raises ImportError with a build hint when it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    L.ibl_version.restype = ctypes.c_int
    L.ibl_last_error.restype = ctypes.c_char_p
    L.ibl_device_count.argtypes = [ctypes.POINTER(_i32)]
    L.ibl_map_node_connections.argtypes = [_i32, _i32, _i32p, _i32p, _i32p, _i32p, _i32p, _i32p, _i32p, _i32p]
    L.ibl_graph_create.argtypes = [_i32, _i32, _i32p, _i32p, _i32, ctypes.POINTER(_vp)]
    L.ibl_graph_info.argtypes = [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i32), ctypes.POINTER(_i64),
                                 ctypes.POINTER(_i32), ctypes.POINTER(_i32)]
    L.ibl_graph_destroy.argtypes = [_vp]
    L.ibl_graph_destroy.restype = None
    L.ibl_ib_create.argtypes = [_vp, _i32, _i32, _i32, _i32p, _i64, _i32p, _i64, _i32p, _i64, _i32p, _i64,
                                _i32, _i32, _i32, ctypes.POINTER(_vp)]
    L.ibl_ib_path.argtypes = [_vp]
    L.ibl_ib_set_path.argtypes = [_vp, _i32]
    L.ibl_ib_path_in_use.argtypes = [_vp, ctypes.POINTER(_i32)]
    L.ibl_ib_fused_ncw.argtypes = [_vp, _i32, ctypes.POINTER(_i32)]
    L.ibl_ib_set_small_batch.argtypes = [_vp, _i32]
    L.ibl_ib_small_batch.argtypes = [_vp, ctypes.POINTER(_i32)]
    L.ibl_ib_decode.argtypes = [_vp, _vp, _i32, _i32, _vp, _i32, _i32, _vp, _vp]
    L.ibl_ib_destroy.argtypes = [_vp]
    L.ibl_ib_destroy.restype = None
    L.ibl_float_create.argtypes = [_vp, _i32, _i32, ctypes.c_double, _i32, _i32, ctypes.POINTER(_vp)]
    L.ibl_float_decode.argtypes = [_vp, _vp, _i32, _i32, _vp, _i32, _i32, _vp, _vp]
    L.ibl_float_destroy.argtypes = [_vp]
    L.ibl_float_destroy.restype = None
    L.ibl_float_set_path.argtypes = [_vp, _i32]
    L.ibl_float_path_in_use.argtypes = [_vp, ctypes.POINTER(_i32)]
    L.ibl_float_folded.argtypes = [_vp, ctypes.POINTER(_i32)]
    L.ibl_float_set_small_batch.argtypes = [_vp, _i32]
    L.ibl_float_small_batch.argtypes = [_vp, ctypes.POINTER(_i32)]
    L.ibl_float_input_check.argtypes = [_vp, ctypes.POINTER(_i32), _vp]
    for nm in ("ibl_ib_timing", "ibl_float_timing"):
        getattr(L, nm).argtypes = [_vp, _i32]
    for nm in ("ibl_ib_timing_read", "ibl_float_timing_read"):
        getattr(L, nm).argtypes = [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i32),
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i32)]
    L.ibl_count_below.argtypes = [_vp, _i32, _i64, _i32, _i64, ctypes.c_double, _vp, _vp]
    _dp = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
    L.ibl_channel_sample.argtypes = [_dp, _i32, _vp, ctypes.c_uint64, ctypes.c_uint64, _i32, _i32, _vp, _vp,
                                     _i32, _i64, _vp]
    L.ibl_encoder_create.argtypes = [_i32, _i32, _i32p, _i32p, _i32, _i32, ctypes.POINTER(_vp)]
    L.ibl_encoder_algorithm.argtypes = [_vp]
    L.ibl_encoder_algorithm.restype = ctypes.c_char_p
    L.ibl_encode.argtypes = [_vp, _vp, _i32, _vp, _vp]
    L.ibl_encoder_destroy.argtypes = [_vp]
    L.ibl_encoder_destroy.restype = None
    L.ibl_random_bits.argtypes = [ctypes.c_uint64, ctypes.c_uint64, _i32, _i32, _vp, _vp]
    L.ibl_count_errors.argtypes = [_vp, _i32, _i64, _i32, _i64, ctypes.c_double, _vp, _i64, _vp, _vp]
    L.ibl_shard_range.argtypes = [_i64, _i32, _i32, ctypes.POINTER(_i64), ctypes.POINTER(_i64)]
    L.ibl_comm_unique_id.argtypes = [_vp]
    L.ibl_comm_create.argtypes = [_vp, _i32, _i32, _i32, ctypes.POINTER(_vp)]
    L.ibl_comm_broadcast.argtypes = [_vp, _vp, _i64, _i32, _vp]
    L.ibl_comm_allreduce_sum_i64.argtypes = [_vp, _vp, _i64, _vp]
    L.ibl_comm_destroy.argtypes = [_vp]
    L.ibl_comm_destroy.restype = None
    for name in EXPORTS:
        getattr(L, name)
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != IBL_OK:
        msg = load().ibl_last_error().decode(errors="replace")
        raise IBLError(f"{what} failed (rc={rc}): {msg}")


def device_count() -> int:
    n = _i32(0)
    load().ibl_device_count(ctypes.byref(n))
    return int(n.value)


def map_node_connections(n_v: int, n_c: int, indptr: np.ndarray, cols: np.ndarray):
    """Host-side index construction through the C ABI (no device needed)."""
    L = load()
    indptr = np.ascontiguousarray(indptr, dtype=np.int32)
    cols = np.ascontiguousarray(cols, dtype=np.int32)
    E = int(indptr[-1])
    cs = np.zeros(n_c, np.int32)
    cd = np.zeros(n_c, np.int32)
    tc = np.zeros(E, np.int32)
    vs = np.zeros(n_v, np.int32)
    vd = np.zeros(n_v, np.int32)
    tv = np.zeros(E, np.int32)
    check(L.ibl_map_node_connections(n_v, n_c, indptr, cols, cs, cd, tc, vs, vd, tv), "ibl_map_node_connections")
    return dict(cn_start=cs, cn_deg=cd, tgt_cn=tc, vn_start=vs, vn_deg=vd, tgt_vn=tv)


def shard_range(total: int, rank: int, world: int):
    """(start, count) of rank's contiguous share of `total` codewords (``ibl_shard_range``; host only)."""
    a, b = _i64(0), _i64(0)
    check(load().ibl_shard_range(int(total), int(rank), int(world), ctypes.byref(a), ctypes.byref(b)), "ibl_shard_range")
    return int(a.value), int(b.value)
