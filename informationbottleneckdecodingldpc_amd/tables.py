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
benchmark use — (b) "LLR-quantised" tables (``T[a,b] = Q(φ(L[a], L[b]))`` with φ the
box-plus / sum of cluster LLRs, one fixed alphabet for every iteration), and (c) since round 6
``de_tables``: discrete density evolution with a message alphabet of its own for every partial node
operation and iteration, and matching vectors between the degrees' alphabets — the structure of the
reference's design (``Discrete_Density_Evolution_irreg.py:75-432``), with each quantiser the
mutual-information-optimal symmetric one on the LLR axis instead of ``lin_sym_sIB``'s search.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

__all__ = [
    "cn_lut_len", "vn_lut_len", "match_cn_len", "match_vn_len",
    "IBTables", "random_tables", "llr_tables", "identity_matching",
    "Alphabet", "de_tables", "edge_degree_distributions",
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


# ------------------------------------------------------------------ discrete density evolution (round 6)
@dataclass
class Alphabet:
    """A message alphabet of T clusters sorted by LLR (cluster t < T/2 <=> LLR < 0 <=> bit 1): the cluster
    probabilities given x = 0 and x = 1 (DE of the all-zero codeword, symmetric decoders) and each cluster's LLR
    log(p0 / p1) (clusters the design leaves empty get a representative LLR that keeps the order)."""
    p0: np.ndarray
    p1: np.ndarray
    L: np.ndarray

    @property
    def T(self) -> int:
        return int(self.L.size)

    def mutual_information(self) -> float:
        return float(_mi_terms(self.p0, self.p1).sum())


_LLR_CAP = 60.0          # cluster LLRs are clipped here (probabilities of ~1e-26): DE stays finite


def _mi_terms(p0, p1):
    """I(X; T) contribution of clusters with p(t | x=0) = p0, p(t | x=1) = p1 and P(x=0) = 1/2."""
    p0 = np.asarray(p0, np.float64)
    p1 = np.asarray(p1, np.float64)
    s = p0 + p1
    with np.errstate(divide="ignore", invalid="ignore"):
        a = np.where(p0 > 0, 0.5 * p0 * np.log2(np.where(p0 > 0, 2 * p0 / np.where(s > 0, s, 1), 1)), 0.0)
        b = np.where(p1 > 0, 0.5 * p1 * np.log2(np.where(p1 > 0, 2 * p1 / np.where(s > 0, s, 1), 1)), 0.0)
    return a + b


def _llr(p0, p1):
    with np.errstate(divide="ignore", invalid="ignore"):
        L = np.log(np.asarray(p0, np.float64)) - np.log(np.asarray(p1, np.float64))
    return np.clip(np.nan_to_num(L, nan=0.0, posinf=_LLR_CAP, neginf=-_LLR_CAP), -_LLR_CAP, _LLR_CAP)


def _boxplus_exact(a, b):
    """LLR of x_a xor x_b from the two LLRs (finite inputs, overflow-free form)."""
    return np.sign(a) * np.sign(b) * np.minimum(np.abs(a), np.abs(b)) + np.log1p(np.exp(-np.abs(a + b))) \
        - np.log1p(np.exp(-np.abs(a - b)))


class _SymQuantiser:
    """The I(X;T)-optimal deterministic symmetric quantiser of outcomes on the LLR axis into T clusters.

    For a binary input the optimal quantiser partitions the outcomes into intervals of their LLR (Kurkoski & Yagi;
    the reference's ``lin_sym_sIB`` searches the same family). With symmetric inputs the outcome set is mirror-
    symmetric, so the T/2 intervals of |LLR| are chosen by dynamic programming over the outcomes sorted by |LLR|
    (outcomes of equal |LLR| kept together), maximising the summed I(X;T) contribution of each interval's
    positive-LLR and negative-LLR halves; interval k is cluster T/2 + k on the positive side and T/2 - 1 - k on the
    negative side (an LLR of exactly 0 counts as positive). ``bounds`` (T/2 - 1 thresholds on |LLR|) map any LLR to
    its cluster, so table entries of zero-probability outcomes follow the same rule."""

    def __init__(self, llr, p0, p1, T):
        llr = np.asarray(llr, np.float64).ravel()
        p0 = np.asarray(p0, np.float64).ravel()
        p1 = np.asarray(p1, np.float64).ravel()
        K = T // 2
        a = np.abs(llr)
        live = (p0 + p1) > 0
        order = np.argsort(a[live], kind="stable")
        av, pos = a[live][order], (llr[live] >= 0)[order]
        q0, q1 = p0[live][order], p1[live][order]
        # groups of equal |LLR| (relative tolerance): one DP unit each
        if av.size:
            brk = np.concatenate([[True], np.diff(av) > 1e-9 * np.maximum(1.0, av[1:])])
            gid = np.cumsum(brk) - 1
        else:
            gid = np.zeros(0, np.int64)
        n = int(gid[-1]) + 1 if gid.size else 0
        gp0 = np.zeros((2, n))
        gp1 = np.zeros((2, n))
        np.add.at(gp0, (pos.astype(int), gid), q0)
        np.add.at(gp1, (pos.astype(int), gid), q1)
        glo = np.full(n, np.inf)
        ghi = np.full(n, -np.inf)
        np.minimum.at(glo, gid, av)
        np.maximum.at(ghi, gid, av)
        c0 = np.concatenate([np.zeros((2, 1)), np.cumsum(gp0, axis=1)], axis=1)
        c1 = np.concatenate([np.zeros((2, 1)), np.cumsum(gp1, axis=1)], axis=1)

        def seg(j, i):      # value of groups j..i-1 as one interval (both sides)
            v = 0.0
            for sd in (0, 1):
                v = v + _mi_terms(c0[sd][i] - c0[sd][j], c1[sd][i] - c1[sd][j])
            return v
        k_used = min(K, n)
        cut = []
        if n:
            jj, ii = np.meshgrid(np.arange(n + 1), np.arange(n + 1), indexing="ij")
            F = seg(jj, ii)
            F = np.where(jj < ii, F, -np.inf)
            best = F[0].copy()                  # one interval over groups 0..i-1
            arg = np.zeros((k_used + 1, n + 1), np.int64)
            for k in range(2, k_used + 1):
                cand = best[:, None] + F        # previous k-1 intervals end at j, interval j..i-1
                arg[k] = np.argmax(cand, axis=0)
                best = cand[arg[k], np.arange(n + 1)]
            i = n
            for k in range(k_used, 1, -1):
                j = int(arg[k][i])
                cut.append(j)
                i = j
            cut = sorted(cut)
        starts = [0] + cut
        ends = cut + [n]
        # |LLR| thresholds between consecutive intervals; clusters past the used ones stay empty
        self.bounds = np.array([0.5 * (ghi[e - 1] + glo[e]) for e in cut], np.float64)
        self.bounds = np.concatenate([self.bounds, np.full(K - 1 - self.bounds.size, np.inf)]) \
            if self.bounds.size < K - 1 else self.bounds
        self.T, self.K = T, K
        P0, P1 = np.zeros(T), np.zeros(T)
        for k, (j, i) in enumerate(zip(starts, ends)):
            P0[K + k], P1[K + k] = c0[1][i] - c0[1][j], c1[1][i] - c1[1][j]
            P0[K - 1 - k], P1[K - 1 - k] = c0[0][i] - c0[0][j], c1[0][i] - c1[0][j]
        # renormalise: every op multiplies two alphabets' masses, so rounding would compound over the iterations
        P0, P1 = P0 / max(P0.sum(), 1e-300), P1 / max(P1.sum(), 1e-300)
        L = _llr(P0, P1)
        # representative LLRs of empty clusters: continue the order beyond the last used interval
        for k in range(K):
            for c, sgn in ((K + k, 1.0), (K - 1 - k, -1.0)):
                if P0[c] + P1[c] <= 0:
                    prev = L[K + k - 1] if sgn > 0 and k > 0 else (L[K - k] if k > 0 else 0.0)
                    L[c] = prev + sgn * 1.0 if k > 0 else sgn * 0.5
        self.alphabet = Alphabet(P0, P1, L)

    def map(self, llr):
        """Cluster of every LLR value (the thresholds of the optimal partition)."""
        llr = np.asarray(llr, np.float64)
        k = np.searchsorted(self.bounds, np.abs(llr), side="left")
        return np.where(llr >= 0, self.K + k, self.K - 1 - k).astype(np.int32)


def _combine(kind, A: Alphabet, Bm: Alphabet):
    """Outcomes (a, b), a-major, of one partial node operation: their p(. | x=0), p(. | x=1) and LLR. kind 'cn':
    x = x_a xor x_b (box-plus); 'vn': x = x_a = x_b (LLRs add)."""
    if kind == "vn":
        p0 = np.outer(A.p0, Bm.p0)
        p1 = np.outer(A.p1, Bm.p1)
        L = A.L[:, None] + Bm.L[None, :]
    else:
        p0 = 0.5 * (np.outer(A.p0, Bm.p0) + np.outer(A.p1, Bm.p1)) * 2.0
        p1 = 0.5 * (np.outer(A.p0, Bm.p1) + np.outer(A.p1, Bm.p0)) * 2.0
        L = _boxplus_exact(A.L[:, None], Bm.L[None, :])
        # p0 / p1 above are p(a, b | x) for uniform independent input bits (sum to 1 over (a, b) each)
        p0, p1 = p0 / 2.0, p1 / 2.0
    live = (p0 + p1) > 0
    Lx = np.where(live, _llr(p0, p1), L)        # exact LLR where the outcome occurs, the node rule elsewhere
    return p0, p1, Lx


def _step(kind, A: Alphabet, Bm: Alphabet, T: int):
    """One partial node operation: the T-cluster table (a-major, [A.T][Bm.T]) and its output alphabet."""
    p0, p1, L = _combine(kind, A, Bm)
    q = _SymQuantiser(L, p0, p1, T)
    return q.map(L), q.alphabet


def _match(outs, weights, T):
    """Common alphabet for the outputs of several node degrees (edge-perspective weights) and each degree's
    matching vector (the reference's information matching, Information_Matching.py:29-71, resolves the degrees'
    'conflicts of opinion' by mapping every degree's clusters onto one alphabet): the optimal symmetric quantiser of
    the pooled clusters, applied to each degree's cluster LLRs."""
    Ls, p0s, p1s = [], [], []
    for A, w in zip(outs, weights):
        Ls.append(A.L)
        p0s.append(w * A.p0)
        p1s.append(w * A.p1)
    tot = float(sum(weights))
    q = _SymQuantiser(np.concatenate(Ls), np.concatenate(p0s) / tot, np.concatenate(p1s) / tot, T)
    return q.alphabet, [q.map(A.L) for A in outs]


def edge_degree_distributions(g):
    """{degree: fraction of edges} of the check and variable sides (the reference's rho / lambda,
    Information_Matching.py:15-26, convert_node_to_edge_degree_from_H)."""
    E = float(np.sum(g.cn_deg))
    rho = {int(d): float(np.sum(g.cn_deg[g.cn_deg == d])) / E for d in np.unique(g.cn_deg)}
    lam = {int(d): float(np.sum(g.vn_deg[g.vn_deg == d])) / E for d in np.unique(g.vn_deg)}
    return rho, lam


def de_tables(p_t_given_x0, L_ch, rho: dict, lam: dict, imax: int, T: int | None = None, match: bool = True,
              return_trace: bool = False):
    """Decoder tables by discrete density evolution with per-iteration message alphabets.

    ``p_t_given_x0`` / ``L_ch``: the channel quantiser's cluster probabilities given bit 0 and cluster LLRs (sorted
    ascending, symmetric: ``channel.UniformQuantizer``); ``rho`` / ``lam``: edge-perspective check / variable degree
    distributions ({degree: fraction}, ``edge_degree_distributions``). Follows the reference's schedule
    (``Discrete_Density_Evolution_irreg.py:75-432``, layout ``Discrete_Density_Evolution.py:299-344``): DE iteration
    i runs the check-node chain — iteration 0 on channel messages (first op channel x channel, ops l >= 1 partial x
    channel, ``kernels_template_irreg.cl:72-81``), later iterations on the previous variable-node output alphabet —
    then the variable-node chain (op 0 channel x check message, ops l >= 1 partial x check message, up to VM - 1 ops
    so the decision over all d inputs has tables, ``:279-300``). Degree d's check output is the chain's alphabet
    after d - 2 ops, its variable output after d - 1 ops; with ``match`` each side's degrees are matched onto one
    common alphabet (the next half iteration's input), without it the alphabets of the most frequent degree stand
    for all. Every op is quantised by ``_SymQuantiser``. Degree-1 variables forward their channel cluster (the
    kernels' rule, no table), so they take no part in the variable-side matching.

    Returns ``IBTables`` (T_ch = T_dec = T), and with ``return_trace`` also the per-iteration mutual information
    I(X; message) of the check and variable outputs."""
    L_ch = np.asarray(L_ch, np.float64)
    Tc = L_ch.size
    T = Tc if T is None else int(T)
    if T != Tc or T % 2:
        raise ValueError("de_tables designs T_dec = T_ch (even)")
    p0c = np.asarray(p_t_given_x0, np.float64)
    p1c = p0c[::-1].copy()                          # symmetric channel: p(t | 1) = p(T-1-t | 0)
    ch = Alphabet(p0c, p1c, _llr(p0c, p1c))
    CM, VM = max(rho), max(lam)
    cdeg = sorted(d for d in rho if rho[d] > 0)
    vdeg = sorted(d for d in lam if lam[d] > 0 and d >= 2)
    cn = np.zeros(cn_lut_len(Tc, T, CM, imax), np.int32)
    vn = np.zeros(vn_lut_len(Tc, T, VM, imax), np.int32)
    mc = identity_matching(T, CM, imax).reshape(imax, CM, T)
    mv = identity_matching(T, VM, imax).reshape(imax, VM, T)
    trace = {"I_cn": [], "I_vn": []}
    V = None
    T2 = T * T
    off_loop = Tc * Tc + (CM - 3) * Tc * T
    for i in range(imax):
        # ---- check-node chain: A_0 = input alphabet, A_{l+1} = Q(A_l x input); degree d outputs A_{d-2}
        inp = ch if i == 0 else V
        A = [inp]
        for l in range(CM - 2):
            if i == 0 and l == 0:
                tab, nxt = _step("cn", ch, ch, T)                     # LUT[m0 * Tc + m1]
                cn[:Tc * Tc] = tab.ravel()
            else:
                tab, nxt = _step("cn", A[-1], inp, T)
                if i == 0:                                          # LUT[Tc^2 + (l-1) Tc T + t T + m] (C6: t*T_dec + y)
                    o = Tc * Tc + (l - 1) * Tc * T
                    cn[o:o + Tc * T] = tab.ravel()[:Tc * T]
                else:                                               # LUT[off + l T^2 + t T + m]
                    o = off_loop + (i - 1) * (CM - 2) * T2 + l * T2
                    cn[o:o + T2] = tab.ravel()
            A.append(nxt)
        outs = [A[d - 2] for d in cdeg]
        if match and len(cdeg) > 1:
            C, maps = _match(outs, [rho[d] for d in cdeg], T)
            for d, m in zip(cdeg, maps):
                mc[i, d - 1] = m
        else:
            C = outs[int(np.argmax([rho[d] for d in cdeg]))]
        trace["I_cn"].append(C.mutual_information())
        # ---- variable-node chain: B_1 = Q(channel x C), B_{l+1} = Q(B_l x C); degree d outputs B_{d-1}
        off = i * (Tc * T + (VM - 1) * T2)
        tab, nxt = _step("vn", ch, C, T)
        vn[off:off + Tc * T] = tab.ravel()
        B = [None, nxt]
        for l in range(1, VM):
            tab, nxt = _step("vn", B[-1], C, T)
            o = off + Tc * T + (l - 1) * T2
            vn[o:o + T2] = tab.ravel()
            B.append(nxt)
        outs = [B[d - 1] for d in vdeg]
        if match and len(vdeg) > 1:
            V, maps = _match(outs, [lam[d] for d in vdeg], T)
            for d, m in zip(vdeg, maps):
                mv[i, d - 1] = m
        else:
            V = outs[int(np.argmax([lam[d] for d in vdeg]))]
        trace["I_vn"].append(V.mutual_information())
    tb = IBTables(Tc, T, CM, VM, imax, cn, vn, mc.ravel().astype(np.int32), mv.ravel().astype(np.int32))
    tb.check()
    return (tb, trace) if return_trace else tb
