"""Parity-check matrices: loaders and generators (reference layer L0).

Everything here is host-side set-up; nothing runs per decoded codeword.

Loaders follow the reference's three on-disk formats
(``Discrete_LDPC_decoding/discrete_LDPC_decoder_irreg.py:102-119``):

* AList text (``alistToNumpy``, ``Discrete_LDPC_decoding/discrete_LDPC_decoder.py:57-81``),
  including the "reduced" AList variant without the weight lines;
* dense ``.npy`` 0/1 matrix (what ``Irregular_LDPC_Decoding/WLAN/generate_802.11_matrix.py:43``
  writes);
* CSR ``.npz`` with keys ``data, indices, indptr, shape``
  (``discrete_LDPC_decoder_irreg.py:102-105``).

Generators (the reference ships no matrices):

* :func:`wlan_80211n` re-implements the quasi-cyclic expansion of
  ``Irregular_LDPC_Decoding/WLAN/generate_802.11_matrix.py:7-34`` (Z=54, N=1296);
  ``Z=81`` uses the standard's own Z=81 rate-1/2 table (:data:`WLAN_R12_BASE_Z81`, N=1944 —
  BASELINE config C3), which the reference does not contain.
* :func:`regular_code` builds a seeded (d_v, d_c)-regular code without double edges,
  standing in for MacKay's ``8000.4000.3.483`` used by
  ``Regular_LDPC_Decoding/BPSK/BER_simulation_OpenCL.py:35``.
* :func:`dvbs2_structured` builds a *DVB-S2-structured* IRA code with the exact R=1/2
  degree profile of ``Irregular_LDPC_Decoding/DVB-S2/decoder_config_generation.py:32-34``
  (synthetic addresses; the EN 302 307 address table is not in the reference).
"""
from __future__ import annotations

import os
from typing import Iterable, Sequence

import numpy as np
import scipy.sparse as sp

__all__ = [
    "alist_to_numpy",
    "load_check_mat",
    "canonical_csr",
    "save_sparse_csr",
    "wlan_80211n",
    "WLAN_R12_BASE",
    "WLAN_R12_BASE_Z81",
    "regular_code",
    "dvbs2_structured",
    "code_rate",
]


def alist_to_numpy(lines: Sequence[Sequence[int]]) -> np.ndarray:
    """AList (list of integer rows) -> dense 0/1 matrix.

    Same contract as ``alistToNumpy`` (``discrete_LDPC_decoder.py:57-81``): line 0 is
    ``nCols nRows``; if lines 2 and 3 have ``nCols`` / ``nRows`` entries they are the
    weight lines and the column lists start at line 4, otherwise at line 2 ("reduced"
    format). Row indices are 1-based, 0 entries are padding.
    """
    n_cols, n_rows = int(lines[0][0]), int(lines[0][1])
    first = 4 if (len(lines[2]) == n_cols and len(lines[3]) == n_rows) else 2
    out = np.zeros((n_rows, n_cols), dtype=np.int64)
    for col in range(n_cols):
        for r in lines[first + col]:
            r = int(r)
            if r != 0:
                out[r - 1, col] = 1
    return out


def _read_alist(filename: str) -> np.ndarray:
    with open(filename) as fh:
        rows = [[int(tok) for tok in line.split()] for line in fh]
    return alist_to_numpy(rows)


def canonical_csr(H) -> sp.csr_matrix:
    """Any 0/1 matrix (dense or sparse) -> CSR with sorted column indices, unit data.

    The reference mixes raw ``H_sparse.indices`` with sorted conversions
    (``discrete_LDPC_decoder_irreg.py:134,146-151``), which is only consistent for a
    canonical CSR; we always canonicalise.
    """
    if sp.issparse(H):
        A = sp.csr_matrix(H, copy=True)
    else:
        A = sp.csr_matrix(np.asarray(H))
    A.sum_duplicates()
    A.eliminate_zeros()
    A.sort_indices()
    A.data = np.ones_like(A.data, dtype=np.int64)
    return A


def load_check_mat(filename: str) -> sp.csr_matrix:
    """Load H from ``.npy`` (dense), ``.npz`` (CSR) or AList text; canonical CSR out."""
    if filename.endswith(".npy"):
        return canonical_csr(np.load(filename, allow_pickle=False))
    if filename.endswith(".npz"):
        with np.load(filename, allow_pickle=False) as z:
            shape = tuple(int(x) for x in z["shape"])
            A = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=shape)
        return canonical_csr(A)
    return canonical_csr(_read_alist(filename))


def save_sparse_csr(filename: str, H) -> None:
    """Write the reference's CSR ``.npz`` layout (``data, indices, indptr, shape``)."""
    A = canonical_csr(H)
    np.savez(filename, data=A.data, indices=A.indices, indptr=A.indptr,
             shape=np.asarray(A.shape))


# IEEE 802.11n rate-1/2 base matrix used by the reference generator
# (generate_802.11_matrix.py:7-19). -1 = all-zero block, s >= 0 = identity rolled by s.
WLAN_R12_BASE = np.array([
    [40, -1, -1, -1, 22, -1, 49, 23, 43, -1, -1, -1, 1, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1],
    [50, 1, -1, -1, 48, 35, -1, -1, 13, -1, 30, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1],
    [39, 50, -1, -1, 4, -1, 2, -1, -1, -1, -1, 49, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1, -1],
    [33, -1, -1, 38, 37, -1, -1, 4, 1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1],
    [45, -1, -1, -1, 0, 22, -1, -1, 20, 42, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1],
    [51, -1, -1, 48, 35, -1, -1, -1, 44, -1, 18, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1],
    [47, 11, -1, -1, -1, 17, -1, -1, 51, -1, -1, -1, 0, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1],
    [5, -1, 25, -1, 6, -1, 45, -1, 13, 40, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1],
    [33, -1, -1, 34, 24, -1, -1, -1, 23, -1, -1, 46, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1],
    [1, -1, 27, -1, 1, -1, -1, -1, 38, -1, 44, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1],
    [-1, 18, -1, -1, 23, -1, -1, 8, 0, 35, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0],
    [49, -1, 17, -1, 30, -1, -1, -1, 34, -1, -1, 19, 1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0],
], dtype=np.int64)


# IEEE 802.11n (802.11-2012 Annex F, Table F.2) rate-1/2 prototype for Z=81 (N=1944), restated
# from the standard: the reference holds only the Z=54 table above, so this table is not pinned by
# a reference output. Structural checks (tests/test_cpu_host.py): the standard's dual-diagonal parity
# part (column 12 shifts 1/0/1), the same column weights as the Z=54 table, and no 4-cycles after
# lifting.
WLAN_R12_BASE_Z81 = np.array([
    [57, -1, -1, -1, 50, -1, 11, -1, 50, -1, 79, -1, 1, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1],
    [3, -1, 28, -1, 0, -1, -1, -1, 55, 7, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1],
    [30, -1, -1, -1, 24, 37, -1, -1, 56, 14, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1, -1],
    [62, 53, -1, -1, 53, -1, -1, 3, 35, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1],
    [40, -1, -1, 20, 66, -1, -1, 22, 28, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1],
    [0, -1, -1, -1, 8, -1, 42, -1, 50, -1, -1, 8, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1],
    [69, 79, 79, -1, -1, -1, 56, -1, 52, -1, -1, -1, 0, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1],
    [65, -1, -1, -1, 38, 57, -1, -1, 72, -1, 27, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1],
    [64, -1, -1, -1, 14, 52, -1, -1, 30, -1, -1, 32, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1],
    [-1, 45, -1, 70, 0, -1, -1, -1, 77, 9, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1],
    [2, 56, -1, 57, 35, -1, -1, -1, -1, -1, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0],
    [24, -1, 61, -1, 60, -1, -1, 27, 51, -1, -1, 16, 1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0],
], dtype=np.int64)


def wlan_80211n(Z: int = 54, base=None) -> sp.csr_matrix:
    """Quasi-cyclic expansion of an 802.11n rate-1/2 prototype with lifting size ``Z``.

    ``base`` defaults to the standard's table for ``Z``: :data:`WLAN_R12_BASE_Z81` for Z=81
    (N=1944), else :data:`WLAN_R12_BASE` (the reference's Z=54 table; other Z give
    WLAN-structured codes). Pass ``base=WLAN_R12_BASE`` to lift the Z=54 table at Z=81.

    Block (i, j) with shift s is the Z×Z identity rolled right by s columns, i.e. row r
    of the block has its 1 in column (r + s) mod Z — the same matrix
    ``np.roll(np.eye(Z), s, axis=1)`` builds in ``generate_802.11_matrix.py:28``.
    Z=54 reproduces the reference's 648×1296 matrix (E=4644).
    """
    if base is None:
        base = WLAN_R12_BASE_Z81 if Z == 81 else WLAN_R12_BASE
    base = np.asarray(base, dtype=np.int64)
    mb, nb = base.shape
    rows, cols = [], []
    r = np.arange(Z)
    for i in range(mb):
        for j in range(nb):
            s = base[i, j]
            if s < 0:
                continue
            rows.append(i * Z + r)
            cols.append(j * Z + (r + s) % Z)
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    H = sp.csr_matrix((np.ones(rows.size, dtype=np.int64), (rows, cols)), shape=(mb * Z, nb * Z))
    return canonical_csr(H)


def regular_code(n: int, dv: int, dc: int, seed: int = 0) -> sp.csr_matrix:
    """Seeded (dv, dc)-regular LDPC code of length n without double edges.

    Socket construction: the n·dv variable sockets are matched to the (n·dv/dc)·dc check
    sockets by a random permutation; any check that received the same variable twice is
    repaired by swapping with a random other socket until every check has dc distinct
    variables.
    """
    if (n * dv) % dc:
        raise ValueError("n*dv must be divisible by dc")
    m = n * dv // dc
    rng = np.random.default_rng(seed)
    var_of_socket = np.repeat(np.arange(n), dv)
    for _ in range(1000):
        perm = rng.permutation(var_of_socket)
        slots = perm.reshape(m, dc)
        for _fix in range(100 * m):
            srt = np.sort(slots, axis=1)
            bad = np.nonzero((srt[:, 1:] == srt[:, :-1]).any(axis=1))[0]
            if bad.size == 0:
                break
            for c in bad:
                row = slots[c]
                vals, counts = np.unique(row, return_counts=True)
                dup = vals[counts > 1][0]
                k = int(np.nonzero(row == dup)[0][0])
                c2 = int(rng.integers(m))
                k2 = int(rng.integers(dc))
                a, b = slots[c, k], slots[c2, k2]
                if b in slots[c] or a in slots[c2]:
                    continue
                slots[c, k], slots[c2, k2] = b, a
        else:
            continue
        rows = np.repeat(np.arange(m), dc)
        H = sp.csr_matrix((np.ones(rows.size, dtype=np.int64), (rows, slots.ravel())), shape=(m, n))
        H = canonical_csr(H)
        if H.nnz == n * dv:
            return H
    raise RuntimeError("could not build a simple regular code")


def dvbs2_structured(seed: int = 0, n: int = 64800, k: int = 32400,
                     groups_hi: int = 36, deg_hi: int = 8, deg_lo: int = 3) -> sp.csr_matrix:
    """DVB-S2-structured IRA code (normal frame, rate 1/2 by default).

    Structure of EN 302 307 §5.3.2: information bits come in groups of 360; group g owns a
    list of addresses x, and bit m of the group connects to check
    ``(x + (m mod 360)·q) mod (n-k)`` with ``q = (n-k)/360``. Parity part is the
    staircase (parity j -> checks j and j+1; the last parity column has degree 1).
    Addresses are synthetic but respect the profile of
    ``DVB-S2/decoder_config_generation.py:32-34``: for the defaults 36 groups of degree 8
    and 54 groups of degree 3, every residue mod q used exactly 5 times, hence check
    degrees {6: 1, 7: 32399} and variable degrees {1: 1, 2: 32399, 3: 19440, 8: 12960},
    E = 226,799.
    """
    m = n - k
    if k % 360 or m % 360:
        raise ValueError("n-k and k must be multiples of 360")
    q = m // 360
    n_groups = k // 360
    degs = [deg_hi] * groups_hi + [deg_lo] * (n_groups - groups_hi)
    total = sum(degs)
    if total % q:
        raise ValueError("address count must be a multiple of q for a check-regular info part")
    rng = np.random.default_rng(seed)
    # residues: each of 0..q-1 used exactly total/q times and no group repeats a residue.
    # Greedy: every group takes the d residues with the most remaining uses (random tie
    # break), which keeps the remaining counts balanced and therefore always feasible.
    remaining = np.full(q, total // q, dtype=np.int64)
    groups = []
    for d in degs:
        key = remaining * 4096 + rng.permutation(q)
        pick = np.argsort(-key, kind="stable")[:d]
        if (remaining[pick] <= 0).any():
            raise RuntimeError("residue assignment failed")
        remaining[pick] -= 1
        groups.append(pick)
    rows, cols = [], []
    mm = np.arange(360)
    for g, resid in enumerate(groups):
        for r in resid:
            x = int(r) + q * int(rng.integers(360))
            rows.append((x + mm * q) % m)
            cols.append(g * 360 + mm)
    # staircase parity part
    j = np.arange(m)
    rows.append(j)
    cols.append(k + j)
    rows.append(j[1:])
    cols.append(k + j[:-1])
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    H = sp.csr_matrix((np.ones(rows.size, dtype=np.int64), (rows, cols)), shape=(m, n))
    H = canonical_csr(H)
    if H.nnz != rows.size:
        raise RuntimeError("duplicate edges in DVB-S2-structured construction")
    return H


def code_rate(H) -> float:
    """Design rate exactly as the reference computes it (float, not K/N).

    ``set_code_parameters`` (``discrete_LDPC_decoder_irreg.py:80-100``): node-perspective
    degree histograms normalised to fractions, R = 1 - <d_v> / <d_c>. For the DVB-S2
    profile this is 0.4999999999999999, so ``data_len = int(R·N) = 32399``;
    keeping the same float arithmetic keeps error counts identical.
    """
    A = canonical_csr(H)
    vdeg = np.asarray(A.sum(0)).ravel()
    cdeg = np.asarray(A.sum(1)).ravel()

    def _mean_from_hist(deg):
        vals = np.unique(deg)
        hist = np.zeros(int(vals.max()))
        for d in np.sort(vals).astype(int):
            hist[d - 1] = (deg == d).sum()
        hist = hist / hist.sum()
        return np.dot(hist, np.arange(vals.max()) + 1)

    return 1 - _mean_from_hist(vdeg) / _mean_from_hist(cdeg)
