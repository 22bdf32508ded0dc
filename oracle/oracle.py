"""ctypes front-end of the CPU oracle (``oracle/ib_oracle.c``).  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import
this module — as the parity checker or the timed CPU baseline. The product package never
imports it and has no CPU fallback.

Arrays follow the reference's layout: channel values / outputs ``[N][B]``; the oracle
restates ``kernels_template_irreg.cl`` and ``kernels_min_and_BP.cl`` (see the C header for
line-level citations).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "ib_oracle.c")
        if not os.path.exists(_LIB_PATH) or (
                os.path.exists(src) and os.path.getmtime(src) > os.path.getmtime(_LIB_PATH)):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i32, i64 = ctypes.c_int32, ctypes.c_int64
        L.ibo_ib_decode.restype = ctypes.c_int
        L.ibo_ib_decode.argtypes = [i32, i32, i64, _i32p, _i32p, _i32p, _i32p, _i32p, _i32p,
                                    i32, i32, i32, i32, i32, _i32p, _i32p, _i32p, _i32p, i32,
                                    _i32p, i32, i32, _i32p, ctypes.POINTER(i32), i32]
        L.ibo_float_decode.restype = ctypes.c_int
        L.ibo_float_decode.argtypes = [i32, i32, i64, _i32p, _i32p, _i32p, _i32p, _i32p, _i32p,
                                       i32, i32, ctypes.c_double, _f64p, i32, i32, _f64p,
                                       ctypes.POINTER(i32), i32]
        L.ibo_max_threads.restype = ctypes.c_int
        for nm in ("ibo_minsum_fold", "ibo_vn_sum"):
            getattr(L, nm).restype = ctypes.c_double
            getattr(L, nm).argtypes = [_f64p, i32]
        L.ibo_boxplus.restype = ctypes.c_double
        L.ibo_boxplus.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double]
        _lib = L
    return _lib


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def ib_decode(g, tb, ch: np.ndarray, match: bool, early_stop: bool = False,
              nthreads: int = 0, return_iters: bool = False):
    """Oracle IB decode of ``ch`` ([N][B] cluster ids) -> [N][B] int32 cluster ids."""
    ch = _c(ch, np.int32)
    if ch.ndim == 1:
        ch = ch[:, None]
    N, B = ch.shape
    assert N == g.n_v
    out = np.zeros((N, B), dtype=np.int32)
    iters = ctypes.c_int32(0)
    rc = lib().ibo_ib_decode(g.n_v, g.n_c, g.n_e, _c(g.cn_start, np.int32), _c(g.cn_deg, np.int32),
                             _c(g.tgt_cn, np.int32), _c(g.vn_start, np.int32), _c(g.vn_deg, np.int32),
                             _c(g.tgt_vn, np.int32), tb.Tc, tb.T, tb.imax, tb.CM, tb.VM,
                             _c(tb.cn, np.int32), _c(tb.vn, np.int32), _c(tb.match_cn, np.int32),
                             _c(tb.match_vn, np.int32), int(bool(match)), ch, B, int(bool(early_stop)),
                             out, ctypes.byref(iters), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle ib_decode failed rc={rc}")
    return (out, iters.value) if return_iters else out


MINSUM, BP = 0, 1


def float_decode(g, kind: int, imax: int, llr: np.ndarray, early_stop: bool = False,
                 llr_max: float = 150.0, nthreads: int = 0, return_iters: bool = False):
    """Oracle fp64 min-sum (kind=0) / BP (kind=1) decode of [N][B] LLRs -> [N][B] APP LLRs."""
    llr = _c(llr, np.float64)
    if llr.ndim == 1:
        llr = llr[:, None]
    N, B = llr.shape
    out = np.zeros((N, B), dtype=np.float64)
    iters = ctypes.c_int32(0)
    rc = lib().ibo_float_decode(g.n_v, g.n_c, g.n_e, _c(g.cn_start, np.int32), _c(g.cn_deg, np.int32),
                                _c(g.tgt_cn, np.int32), _c(g.vn_start, np.int32), _c(g.vn_deg, np.int32),
                                _c(g.tgt_vn, np.int32), int(kind), int(imax), float(llr_max), llr, B,
                                int(bool(early_stop)), out, ctypes.byref(iters), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle float_decode failed rc={rc}")
    return (out, iters.value) if return_iters else out


def max_threads() -> int:
    return int(lib().ibo_max_threads())


def minsum_fold(m) -> float:
    m = _c(m, np.float64)
    return float(lib().ibo_minsum_fold(m, m.size))


def vn_sum(m) -> float:
    m = _c(m, np.float64)
    return float(lib().ibo_vn_sum(m, m.size))


def boxplus(a: float, b: float, llr_max: float = 150.0) -> float:
    return float(lib().ibo_boxplus(a, b, llr_max))
