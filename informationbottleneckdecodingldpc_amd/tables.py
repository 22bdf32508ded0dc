"""IB decoder lookup tables: reference layout, validation, and generators.

Layout (the output of the reference's discrete density evolution, consumed by
``kernels_template[_irreg].cl``). ``T = T_dec``, ``Tc = T_ch``,
``CM = d_c_max``, ``VM = d_v_max``, ``I = i_max``:

* CN vector, length ``Tc² + (CM-3)·Tc·T + (I-1)·(CM-2)·T²``
  (``Discrete_LDPC_decoding/Discrete_Density_Evolution.py:92-95``, filled ``:299-324``):
  iteration-0 ops first (``kernels_template_irreg.cl:72-81``), then ``I-1`` loop passes of
  ``CM-2`` blocks of ``T²`` (``:205-231``).
* VN vector, length ``I·(Tc·T + (VM-1)·T²)`` (``Discrete_Density_Evolution.py:120-122``):
  per pass a ``Tc·T`` channel block and ``VM-1`` message blocks (``:328-344``).
* Matching vectors (irregular decoder with ``match='true'``): CN ``(I, CM, T)`` and VN
  ``(I, VM, T)`` C-order (``Discrete_Density_Evolution_irreg.py:49,431``), read at
  ``(pass)·T·CM + (d-1)·T + t`` (``kernels_template_irreg.cl:84-91,233-240,162-172``).

The reference obtains table *values* from the information-bottleneck design in the
absent ``ib_base`` package. This module provides (a) uniformly random
tables — the decode work is value-independent, so they are what parity tests and the
benchmark use — and (b) "LLR-quantised" tables (``T[a,b] = Q(φ(L[a], L[b]))`` with φ the
box-plus / sum of cluster LLRs) that decode well enough for meaningful BER curves.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

__all__ = [
    "cn_lut_len", "vn_lut_len", "match_cn_len", "match_vn_len",
    "IBTables", "random_tables", "llr_tables", "identity_matching",
]


def cn_lut_len(Tc: int, T: int, CM: int, imax: int) -> int:
    return Tc * Tc + (CM - 3) * Tc * T + (imax - 1) * (CM - 2) * T * T


def vn_lut_len(Tc: int, T: int, VM: int, imax: int) -> int:
    return imax * (Tc * T + (VM - 1) * T * T)


def match_cn_len(T: int, CM: int, imax: int) -> int:
    return imax * CM * T


def match_vn_len(T: int, VM: int, imax: int) -> int:
    return imax * VM * T


@dataclass
class IBTables:
    Tc: int
    T: int
    CM: int
    VM: int
    imax: int
    cn: np.ndarray            # int32 flat CN LUT vector
    vn: np.ndarray            # int32 flat VN LUT vector
    match_cn: np.ndarray      # int32 flat (imax, CM, T)
    match_vn: np.ndarray      # int32 flat (imax, VM, T)

    def check(self) -> None:
        want = (cn_lut_len(self.Tc, self.T, self.CM, self.imax),
                vn_lut_len(self.Tc, self.T, self.VM, self.imax))
        if self.cn.size < want[0] or self.vn.size < want[1]:
            raise ValueError(f"LUT vectors too short: got {(self.cn.size, self.vn.size)}, need {want}")
        for name, v in (("cn", self.cn), ("vn", self.vn), ("match_cn", self.match_cn),
                        ("match_vn", self.match_vn)):
            if v.size and (v.min() < 0 or v.max() >= self.T):
                raise ValueError(f"{name} entries must lie in [0, T_dec)")


def identity_matching(T: int, D: int, imax: int) -> np.ndarray:
    return np.tile(np.arange(T, dtype=np.int32), imax * D)


def random_tables(Tc: int, T: int, CM: int, VM: int, imax: int, seed: int = 1,
                  random_matching: bool = True) -> IBTables:
    """Uniform random tables in [0, T) of exactly the reference lengths (parity / bench)."""
    rng = np.random.default_rng(seed)
    cn = rng.integers(0, T, cn_lut_len(Tc, T, CM, imax), dtype=np.int32)
    vn = rng.integers(0, T, vn_lut_len(Tc, T, VM, imax), dtype=np.int32)
    if random_matching:
        mc = rng.integers(0, T, match_cn_len(T, CM, imax), dtype=np.int32)
        mv = rng.integers(0, T, match_vn_len(T, VM, imax), dtype=np.int32)
    else:
        mc = identity_matching(T, CM, imax)
        mv = identity_matching(T, VM, imax)
    return IBTables(Tc, T, CM, VM, imax, cn, vn, mc, mv)


def _boxplus(a, b):
    s = np.sign(a) * np.sign(b)
    return s * np.minimum(np.abs(a), np.abs(b)) + np.log1p(np.exp(-np.abs(a + b))) \
        - np.log1p(np.exp(-np.abs(a - b)))


def _quantise(x: np.ndarray, L: np.ndarray) -> np.ndarray:
    """Nearest cluster (in LLR) of x among the sorted representative LLRs L."""
    mid = 0.5 * (L[1:] + L[:-1])
    return np.searchsorted(mid, x).astype(np.int32)


def llr_tables(L_ch: np.ndarray, CM: int, VM: int, imax: int, scale: float = 1.0,
               T: int | None = None) -> IBTables:
    """Tables that approximate BP on cluster LLRs (not information-optimal, but decoding).

    ``L_ch[t]`` are the channel clusters' LLRs sorted ascending (cluster ``t < T/2`` ⇒
    negative LLR ⇒ bit 1, matching the reference's decision ``t < T/2``). The decoder's
    message alphabet reuses the same representative values, optionally scaled.
    """
    L_ch = np.asarray(L_ch, dtype=np.float64)
    Tc = L_ch.size
    T = Tc if T is None else T
    Ld = np.sort(L_ch)[np.linspace(0, Tc - 1, T).round().astype(int)] * scale
    a = np.arange
    cn0 = _quantise(_boxplus(L_ch[:, None], L_ch[None, :]), Ld).ravel()          # Tc x Tc
    cn0t = _quantise(_boxplus(Ld[:, None], L_ch[None, :]), Ld).ravel()           # T x Tc blocks
    cnl = _quantise(_boxplus(Ld[:, None], Ld[None, :]), Ld).ravel()              # T x T
    # iteration-0 op l>=1 indexes t*T + y (kernels_template_irreg.cl:77) with block Tc*T
    blk0 = np.zeros(Tc * T, dtype=np.int32)
    idx = (a(T)[:, None] * T + a(Tc)[None, :]).ravel()
    ok = idx < Tc * T
    blk0[idx[ok]] = cn0t[ok]
    cn = np.concatenate([cn0] + [blk0] * (CM - 3) + [cnl] * ((imax - 1) * (CM - 2))).astype(np.int32)
    vch = _quantise(L_ch[:, None] + Ld[None, :], Ld).ravel()                      # Tc x T
    vl = _quantise(Ld[:, None] + Ld[None, :], Ld).ravel()                         # T x T
    vn = np.concatenate(([vch] + [vl] * (VM - 1)) * imax).astype(np.int32)
    return IBTables(Tc, T, CM, VM, imax, cn, vn, identity_matching(T, CM, imax),
                    identity_matching(T, VM, imax))
