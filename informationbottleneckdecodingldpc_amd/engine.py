"""Device-side decoder objects over the C ABI (torch tensors as device memory, HIP streams).

These are the building blocks of the reference-compatible classes
(:mod:`.discrete_LDPC_decoder`, :mod:`.discrete_LDPC_decoder_irreg`,
:mod:`.min_sum_decoder_irreg`, :mod:`.bp_decoder_irreg`). PyTorch is only plumbing:
allocation, streams and ``torch.distributed``; every decode runs the HIP kernels of
``libibldpc.so`` and there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from . import _lib
from .graph import EdgeGraph, build_graph
from .tables import IBTables

_DT_IB = {torch.uint8: _lib.IBL_U8, torch.int32: _lib.IBL_I32}
_DT_FL = {torch.float32: _lib.IBL_F32, torch.float64: _lib.IBL_F64}
_DT_ANY = {torch.uint8: _lib.IBL_U8, torch.int32: _lib.IBL_I32, torch.float32: _lib.IBL_F32,
           torch.float64: _lib.IBL_F64}


def _require_gpu(device) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible: the LDPC decoders run only on the GPU (no CPU fallback)")
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if dev.type != "cuda":
        raise ValueError(f"decoder device must be a HIP (cuda) device, got {dev}")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def _stream_ptr(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _check_tensor(t: torch.Tensor, dev: torch.device, n_rows: int, name: str) -> None:
    if not isinstance(t, torch.Tensor) or t.device != dev:
        raise ValueError(f"{name} must be a tensor on {dev}")
    if t.dim() != 2 or t.shape[0] != n_rows or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous [{n_rows}][B] tensor, got {tuple(t.shape)}")


class Graph:
    """A code graph uploaded to one device (``ibl_graph``)."""

    def __init__(self, H_or_graph, device=None):
        self.device = _require_gpu(device)
        self.edges: EdgeGraph = H_or_graph if isinstance(H_or_graph, EdgeGraph) else build_graph(H_or_graph)
        g = self.edges
        L = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(L.ibl_graph_create(g.n_v, g.n_c, np.ascontiguousarray(g.csr_indptr, np.int32),
                                      np.ascontiguousarray(g.csr_cols, np.int32), self.device.index,
                                      ctypes.byref(h)), "ibl_graph_create")
        self._h = h

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.load().ibl_graph_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self._h = None


class IBDecoder:
    """Information-bottleneck lookup-table decoder (``ibl_ib``) for up to ``max_batch`` codewords.

    ``path`` (fast path only): "auto" (the fused on-chip kernel when the code fits in LDS), "passes"
    (one launch per check / variable pass) or "fused" (raises when the code does not fit); both give
    identical results (``ibl_ib_set_path``). ``fused`` tells which one decodes run."""

    _PATHS = {"auto": _lib.IBL_PATH_AUTO, "passes": _lib.IBL_PATH_PASSES, "fused": _lib.IBL_PATH_FUSED}

    def __init__(self, graph: Graph, tables: IBTables, match: bool, max_batch: int, force_generic: bool = False,
                 path: str = "auto"):
        self.graph = graph
        self.tables = tables
        self.match = bool(match)
        self.max_batch = int(max_batch)
        self.device = graph.device
        tb = tables
        cn = np.ascontiguousarray(tb.cn, np.int32)
        vn = np.ascontiguousarray(tb.vn, np.int32)
        mc = np.ascontiguousarray(tb.match_cn if tb.match_cn is not None else np.zeros(1), np.int32)
        mv = np.ascontiguousarray(tb.match_vn if tb.match_vn is not None else np.zeros(1), np.int32)
        h = ctypes.c_void_p()
        L = _lib.load()
        _lib.check(L.ibl_ib_create(graph.handle, tb.Tc, tb.T, tb.imax, cn, cn.size, vn, vn.size, mc, mc.size,
                                   mv, mv.size, int(self.match), self.max_batch,
                                   _lib.IBL_FLAG_FORCE_GENERIC if force_generic else 0, ctypes.byref(h)),
                   "ibl_ib_create")
        self._h = h
        self.fast_path = bool(L.ibl_ib_path(h))
        if path not in self._PATHS:
            raise ValueError(f"path must be one of {sorted(self._PATHS)}")
        _lib.check(L.ibl_ib_set_path(h, self._PATHS[path]), "ibl_ib_set_path")

    @property
    def fused(self) -> bool:
        f = ctypes.c_int32()
        _lib.check(_lib.load().ibl_ib_path_in_use(self._h, ctypes.byref(f)), "ibl_ib_path_in_use")
        return bool(f.value)

    @property
    def small_batch(self) -> int:
        """Largest batch the small-batch kernels decode (``ibl_ib_small_batch``; 0 = off)."""
        n = ctypes.c_int32()
        _lib.check(_lib.load().ibl_ib_small_batch(self._h, ctypes.byref(n)), "ibl_ib_small_batch")
        return int(n.value)

    @small_batch.setter
    def small_batch(self, max_b: int) -> None:
        _lib.check(_lib.load().ibl_ib_set_small_batch(self._h, int(max_b)), "ibl_ib_set_small_batch")

    def fused_ncw(self, B: int) -> int:
        """Codewords per workgroup the fused kernel decodes a batch of ``B`` with (8, or 4 for half
        groups; 0 when the fused kernel is not in use) — ``ibl_ib_fused_ncw``."""
        n = ctypes.c_int32()
        _lib.check(_lib.load().ibl_ib_fused_ncw(self._h, int(B), ctypes.byref(n)), "ibl_ib_fused_ncw")
        return int(n.value)

    def decode(self, ch: torch.Tensor, out: Optional[torch.Tensor] = None, out_dtype=torch.int32,
               early_stop: bool = True, iters: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Decode ``ch`` ([N][B] cluster ids, uint8/int32, on the decoder's device)."""
        n = self.graph.edges.n_v
        _check_tensor(ch, self.device, n, "channel values")
        if ch.dtype not in _DT_IB:
            raise ValueError("channel values must be uint8 or int32")
        B = ch.shape[1]
        if out is None:
            out = torch.empty((n, B), dtype=out_dtype, device=self.device)
        _check_tensor(out, self.device, n, "output")
        if out.dtype not in _DT_IB or out.shape[1] != B:
            raise ValueError("output must be uint8/int32 [N][B]")
        it_ptr = None
        if iters is not None:
            if iters.dtype != torch.int32 or iters.device != self.device or iters.numel() < 1:
                raise ValueError("iters must be an int32 device tensor")
            it_ptr = iters.data_ptr()
        _lib.check(_lib.load().ibl_ib_decode(self._h, ch.data_ptr(), _DT_IB[ch.dtype], B, out.data_ptr(),
                                             _DT_IB[out.dtype], int(bool(early_stop)), it_ptr,
                                             _stream_ptr(self.device)), "ibl_ib_decode")
        return out

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.load().ibl_ib_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self._h = None


class FloatDecoder:
    """Float min-sum (kind=0) / BP (kind=1) decoder (``ibl_float``); precision fp32 or fp64.

    ``path``: "auto" (the fused on-chip kernel when the code fits in LDS), "passes" (one launch per
    check / variable pass) or "fused" (raises when the code does not fit); both give identical
    results (``ibl_float_set_path``). ``fused`` tells which one decodes run."""

    _PATHS = {"auto": _lib.IBL_PATH_AUTO, "passes": _lib.IBL_PATH_PASSES, "fused": _lib.IBL_PATH_FUSED}

    def __init__(self, graph: Graph, kind: int, imax: int, max_batch: int, precision=torch.float32,
                 llr_max: float = 150.0, path: str = "auto"):
        self.graph = graph
        self.kind = int(kind)
        self.imax = int(imax)
        self.max_batch = int(max_batch)
        self.precision = precision
        self.device = graph.device
        h = ctypes.c_void_p()
        _lib.check(_lib.load().ibl_float_create(graph.handle, self.kind, self.imax, float(llr_max),
                                                _DT_FL[precision], self.max_batch, ctypes.byref(h)),
                   "ibl_float_create")
        self._h = h
        if path not in self._PATHS:
            raise ValueError(f"path must be one of {sorted(self._PATHS)}")
        _lib.check(_lib.load().ibl_float_set_path(h, self._PATHS[path]), "ibl_float_set_path")

    @property
    def fused(self) -> bool:
        f = ctypes.c_int32()
        _lib.check(_lib.load().ibl_float_path_in_use(self._h, ctypes.byref(f)), "ibl_float_path_in_use")
        return bool(f.value)

    @property
    def small_batch(self) -> int:
        """Largest batch the small-batch float kernels decode (``ibl_float_small_batch``; 0 = off)."""
        n = ctypes.c_int32()
        _lib.check(_lib.load().ibl_float_small_batch(self._h, ctypes.byref(n)), "ibl_float_small_batch")
        return int(n.value)

    @small_batch.setter
    def small_batch(self, max_b: int) -> None:
        _lib.check(_lib.load().ibl_float_set_small_batch(self._h, int(max_b)), "ibl_float_set_small_batch")

    @property
    def folded(self) -> int:
        """Degree-2 variables the per-pass path folds into the check pass (``ibl_float_folded``)."""
        f = ctypes.c_int32()
        _lib.check(_lib.load().ibl_float_folded(self._h, ctypes.byref(f)), "ibl_float_folded")
        return int(f.value)

    def input_violations(self, raise_on_error: bool = True) -> int:
        """Channel LLRs of this decoder's decodes since the last call (on any stream) that broke the
        precondition (NaN; BP fp64 also |x| > 709.78, BP fp32 also +-inf): synchronises the device and clears
        the count (``ibl_float_input_check``). Raises :class:`_lib.IBLError` when there were any, unless
        ``raise_on_error`` is False."""
        v = ctypes.c_int32()
        rc = _lib.load().ibl_float_input_check(self._h, ctypes.byref(v), _stream_ptr(self.device))
        if raise_on_error:
            _lib.check(rc, "ibl_float_input_check")
        return int(v.value)

    def decode(self, llr: torch.Tensor, out: Optional[torch.Tensor] = None, out_dtype=None,
               early_stop: bool = True, iters: Optional[torch.Tensor] = None) -> torch.Tensor:
        n = self.graph.edges.n_v
        _check_tensor(llr, self.device, n, "channel LLRs")
        if llr.dtype not in _DT_FL:
            raise ValueError("channel LLRs must be float32 or float64")
        B = llr.shape[1]
        if out is None:
            out = torch.empty((n, B), dtype=out_dtype or self.precision, device=self.device)
        _check_tensor(out, self.device, n, "output")
        if out.dtype not in _DT_FL or out.shape[1] != B:
            raise ValueError("output must be float32/float64 [N][B]")
        it_ptr = None
        if iters is not None:
            if iters.dtype != torch.int32 or iters.device != self.device or iters.numel() < 1:
                raise ValueError("iters must be an int32 device tensor")
            it_ptr = iters.data_ptr()
        _lib.check(_lib.load().ibl_float_decode(self._h, llr.data_ptr(), _DT_FL[llr.dtype], B, out.data_ptr(),
                                                _DT_FL[out.dtype], int(bool(early_stop)), it_ptr,
                                                _stream_ptr(self.device)), "ibl_float_decode")
        return out

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.load().ibl_float_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self._h = None


def count_below(x: torch.Tensor, rows: int, threshold: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Device count of ``x[:rows] < threshold`` (the reference's error counters) -> int64 tensor."""
    if x.dim() != 2 or not x.is_contiguous() or x.device.type != "cuda":
        raise ValueError("x must be a contiguous 2-D device tensor")
    if x.dtype not in _DT_ANY:
        raise ValueError("unsupported dtype")
    if out is None:
        out = torch.empty(1, dtype=torch.int64, device=x.device)
    rows = min(int(rows), x.shape[0])
    _lib.check(_lib.load().ibl_count_below(x.data_ptr(), _DT_ANY[x.dtype], rows, x.shape[1], x.shape[1],
                                           float(threshold), out.data_ptr(), _stream_ptr(x.device)),
               "ibl_count_below")
    return out


def philox_blocks(n: int, B: int) -> int:
    """Philox counter blocks one channel batch of n*B values consumes (4 values per block)."""
    return (int(n) * int(B) + 3) // 4


def channel_sample(out: torch.Tensor, cdf: np.ndarray, seed: int, offset: int,
                   llr: Optional[np.ndarray] = None, bits: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Direct-inversion channel samples on the device (``ibl_channel_sample``; the reference's
    ``quantize_direct_OpenCL`` / ``quantize_direct_OpenCL_LLR``, AWGN_Quantizer_BPSK.py:216-260).

    ``out``: contiguous [n][B] device tensor — uint8 / int32 receive cluster ids, float32 / float64
    receive ``llr[cluster]``. ``cdf``: the quantiser's T+1 CDF of p(t | x = 0). Uniforms come from
    numpy-compatible Philox4x64-10 (counter ``offset``, key ``seed``); the batch consumes
    :func:`philox_blocks` counter blocks. ``bits`` (optional [n][B] uint8 device tensor): codeword
    bits, 1 mirrors the cluster."""
    if out.dim() != 2 or not out.is_contiguous() or out.device.type != "cuda":
        raise ValueError("out must be a contiguous 2-D device tensor")
    if out.dtype not in _DT_ANY:
        raise ValueError("out dtype must be uint8, int32, float32 or float64")
    cdf = np.ascontiguousarray(cdf, dtype=np.float64)
    T = len(cdf) - 1
    llr_arr = None
    if out.dtype in _DT_FL:
        if llr is None or len(llr) != T:
            raise ValueError("LLR output needs llr with T entries")
        llr_arr = np.ascontiguousarray(llr, dtype=np.float64)
    n, B = out.shape
    bptr = None
    if bits is not None:
        if bits.dtype != torch.uint8 or bits.shape != out.shape or not bits.is_contiguous() or bits.device != out.device:
            raise ValueError("bits must be a contiguous uint8 tensor shaped like out, on the same device")
        bptr = bits.data_ptr()
    _lib.check(_lib.load().ibl_channel_sample(cdf, T, None if llr_arr is None else llr_arr.ctypes.data,
                                              int(seed) & (2 ** 64 - 1), int(offset) & (2 ** 64 - 1), n, B, bptr,
                                              out.data_ptr(), _DT_ANY[out.dtype], B, _stream_ptr(out.device)),
               "ibl_channel_sample")
    return out


class Encoder:
    """Batched systematic LDPC encoder on one device (``ibl_encoder``; the reference's
    Discrete_LDPC_decoding/LDPC_encoder.py plan :197-269 and encode :86-123, for B words at once)."""

    def __init__(self, H, max_batch: int, device=None):
        from .codes import canonical_csr
        self.device = _require_gpu(device)
        Hc = canonical_csr(H)
        self.N_c, self.N = Hc.shape
        self.K = self.N - self.N_c
        self.max_batch = int(max_batch)
        h = ctypes.c_void_p()
        _lib.check(_lib.load().ibl_encoder_create(self.N, self.N_c, np.ascontiguousarray(Hc.indptr, np.int32),
                                                  np.ascontiguousarray(Hc.indices, np.int32), self.max_batch,
                                                  self.device.index, ctypes.byref(h)), "ibl_encoder_create")
        self._h = h
        self.algorithm = _lib.load().ibl_encoder_algorithm(h).decode()

    def encode(self, info: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """u8 [K][B] information bits on the device -> u8 [N][B] codewords [info; parity]."""
        _check_tensor(info, self.device, self.K, "info")
        if info.dtype != torch.uint8:
            raise ValueError("info must be uint8")
        B = info.shape[1]
        if out is None:
            out = torch.empty((self.N, B), dtype=torch.uint8, device=self.device)
        _check_tensor(out, self.device, self.N, "out")
        if out.dtype != torch.uint8 or out.shape[1] != B:
            raise ValueError("out must be a uint8 [N][B] tensor")
        _lib.check(_lib.load().ibl_encode(self._h, info.data_ptr(), B, out.data_ptr(), _stream_ptr(self.device)),
                   "ibl_encode")
        return out

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.load().ibl_encoder_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self._h = None


def random_bits(out: torch.Tensor, seed: int, offset: int) -> torch.Tensor:
    """Fill a contiguous u8 [n][B] device tensor with information bits from the numpy-compatible
    Philox4x64-10 stream (top bit of each output; consumes :func:`philox_blocks` counter blocks)."""
    if out.dim() != 2 or not out.is_contiguous() or out.device.type != "cuda" or out.dtype != torch.uint8:
        raise ValueError("out must be a contiguous 2-D uint8 device tensor")
    n, B = out.shape
    _lib.check(_lib.load().ibl_random_bits(int(seed) & (2 ** 64 - 1), int(offset) & (2 ** 64 - 1), n, B,
                                           out.data_ptr(), _stream_ptr(out.device)), "ibl_random_bits")
    return out


def count_errors(x: torch.Tensor, rows: int, threshold: float, bits: torch.Tensor,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Device count of decided bits ``x[:rows] < threshold`` that differ from ``bits[:rows]`` -> int64."""
    if x.dim() != 2 or not x.is_contiguous() or x.device.type != "cuda" or x.dtype not in _DT_ANY:
        raise ValueError("x must be a contiguous 2-D device tensor (uint8/int32/float32/float64)")
    if bits.dtype != torch.uint8 or bits.dim() != 2 or not bits.is_contiguous() or bits.device != x.device \
            or bits.shape[1] != x.shape[1]:
        raise ValueError("bits must be a contiguous uint8 [n][B] tensor on x's device")
    rows = min(int(rows), x.shape[0], bits.shape[0])
    if out is None:
        out = torch.empty(1, dtype=torch.int64, device=x.device)
    _lib.check(_lib.load().ibl_count_errors(x.data_ptr(), _DT_ANY[x.dtype], rows, x.shape[1], x.shape[1],
                                            float(threshold), bits.data_ptr(), bits.shape[1], out.data_ptr(),
                                            _stream_ptr(x.device)), "ibl_count_errors")
    return out
