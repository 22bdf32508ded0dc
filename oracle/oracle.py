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
        srcs = [os.path.join(_HERE, f) for f in ("ib_oracle.c", "float_oracle.inc", "channel_oracle.c", "Makefile")]
        if not os.path.exists(_LIB_PATH) or any(
                os.path.exists(src) and os.path.getmtime(src) > os.path.getmtime(_LIB_PATH) for src in srcs):
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
        _f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
        L.ibo_float32_decode.restype = ctypes.c_int
        L.ibo_float32_decode.argtypes = [i32, i32, i64, _i32p, _i32p, _i32p, _i32p, _i32p, _i32p,
                                         i32, i32, ctypes.c_float, _f32p, i32, i32, _f32p,
                                         ctypes.POINTER(i32), ctypes.c_void_p, i32]
        L.ibo_max_threads.restype = ctypes.c_int
        for nm in ("ibo_minsum_fold", "ibo_vn_sum"):
            getattr(L, nm).restype = ctypes.c_double
            getattr(L, nm).argtypes = [_f64p, i32]
        L.ibo_boxplus.restype = ctypes.c_double
        L.ibo_boxplus.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double]
        _u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
        _u8p = ctypes.c_void_p
        L.ibo_philox_raw.argtypes = [_u64p, _u64p, i64, _u64p]
        L.ibo_invert_cdf.argtypes = [_f64p, i64, _f64p, i32, _u8p, _i32p]
        L.ibo_channel_sample.argtypes = [_f64p, i32, ctypes.c_uint64, ctypes.c_uint64, i64, _u8p, _i32p]
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


def float32_decode(g, imax: int, llr: np.ndarray, early_stop: bool = False, llr_max: float = 150.0,
                   nthreads: int = 0, return_iters: bool = False, return_syndromes: bool = False):
    """Oracle fp32 min-sum decode (the exact float32 restatement: same operations in the same order
    as kernels_min_and_BP.cl, IEEE single arithmetic) of [N][B] float32 LLRs -> [N][B] float32.
    return_syndromes adds the syndrome sum after every loop iteration (index i = iteration i,
    -1 where none ran)."""
    llr = _c(llr, np.float32)
    if llr.ndim == 1:
        llr = llr[:, None]
    N, B = llr.shape
    out = np.zeros((N, B), dtype=np.float32)
    iters = ctypes.c_int32(0)
    syn = np.zeros(max(int(imax), 1), dtype=np.int64)
    rc = lib().ibo_float32_decode(g.n_v, g.n_c, g.n_e, _c(g.cn_start, np.int32), _c(g.cn_deg, np.int32),
                                  _c(g.tgt_cn, np.int32), _c(g.vn_start, np.int32), _c(g.vn_deg, np.int32),
                                  _c(g.tgt_vn, np.int32), MINSUM, int(imax), float(llr_max), llr, B,
                                  int(bool(early_stop)), out, ctypes.byref(iters),
                                  syn.ctypes.data if return_syndromes else None, int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle float32_decode failed rc={rc}")
    res = (out,)
    if return_iters:
        res += (iters.value,)
    if return_syndromes:
        res += (syn,)
    return res if len(res) > 1 else out


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


# ---------------------------------------------------------------- channel generation
def philox_raw(counter: int, key: int, count: int) -> np.ndarray:
    """First `count` 64-bit outputs of Philox4x64-10 in numpy's stream layout
    (np.random.Philox(counter=counter, key=key).random_raw(count))."""
    ctr = np.array([(counter >> (64 * i)) & (2 ** 64 - 1) for i in range(4)], dtype=np.uint64)
    k = np.array([(key >> (64 * i)) & (2 ** 64 - 1) for i in range(2)], dtype=np.uint64)
    out = np.zeros(count, np.uint64)
    lib().ibo_philox_raw(ctr, k, count, out)
    return out


def invert_cdf(u: np.ndarray, cdf: np.ndarray, bits: np.ndarray | None = None) -> np.ndarray:
    """Reference direct-inversion rule (kernels_quanti_template.cl:19-28; bit 1 mirrors,
    AWGN_Quantizer_BPSK.py:137-143): t = #{w in 1..T: u > cdf[w]} (t = T clamped to T-1)."""
    u = _c(u, np.float64)
    cdf = _c(cdf, np.float64)
    out = np.zeros(u.shape, np.int32)
    b = None if bits is None else np.ascontiguousarray(bits, dtype=np.uint8)
    lib().ibo_invert_cdf(u.ravel(), u.size, cdf, len(cdf) - 1, None if b is None else b.ctypes.data,
                         out.reshape(-1))
    return out


def channel_sample(cdf: np.ndarray, seed: int, offset: int, n: int, B: int,
                   bits: np.ndarray | None = None) -> np.ndarray:
    """ibl_channel_sample restated: [n][B] int32 cluster ids."""
    cdf = _c(cdf, np.float64)
    out = np.zeros((n, B), np.int32)
    b = None if bits is None else np.ascontiguousarray(bits, dtype=np.uint8)
    lib().ibo_channel_sample(cdf, len(cdf) - 1, seed, offset, n * B, None if b is None else b.ctypes.data, out)
    return out


def random_bits(seed: int, offset: int, n: int, B: int) -> np.ndarray:
    """u8 [n][B] information bits of ibl_random_bits: top bit of each 64-bit output of numpy's
    Philox4x64-10 stream with key (seed, 1) — key word 1 set, so the stream is disjoint from the
    channel's key (seed, 0) — and counter offset (the stand-in for LDPC_Transmitter.py:111's
    np.random.randint(0, 2, (data_len, msg_at_time)))."""
    key = (int(seed) & (2 ** 64 - 1)) | (1 << 64)
    return (philox_raw(int(offset), key, int(n) * int(B)) >> np.uint64(63)).astype(np.uint8).reshape(n, B)
