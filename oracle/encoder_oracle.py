"""CPU ORACLE for the LDPC encoder (TEST INFRASTRUCTURE ONLY — same rules as ib_oracle.c: only
tests/, smoke() and bench.py's cpu_baseline leg use it).

Restates the reference's Discrete_LDPC_decoding/LDPC_encoder.py for a batch of information words:
  getLDPCEncoderParamters (:197-269)  H = [A | B]; B triangular with full diagonal -> forward (lower)
                                      or backward (upper) substitution, also after reversing B's rows
                                      (row order), else GF(2) factorisation B = L * U (gf2factorize
                                      :287-340) with pivot row order
  encode (:86-123)                    r = A x; [L substitution]; [r = r[row_order]]; substitution with
                                      the strictly triangular part P; codeword = [x; p]
GF2MatrixMul (:164-190) runs column by column in place; because L and P are strictly triangular that
equals the row-oriented recurrences used here (p_i = r_i xor XOR_{j: P[i,j]} p_j in substitution
order). Pinned by tests/golden/reference_encoder.npz (the reference's own encode on seeded words).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def _is_full_diag_triangular(X: sp.spmatrix) -> int:
    """1 lower / -1 upper triangular with a full diagonal, else 0 (isfulldiagtriangular :342-360)."""
    X = sp.csr_matrix(X)
    if not np.all(X.diagonal() != 0):
        return 0
    nnz = (X != 0).sum()
    low = (sp.tril(X) != 0).sum()
    if low == nnz:
        return 1
    if low == X.shape[0]:
        return -1
    return 0


def gf2factorize(X: np.ndarray):
    """Gaussian elimination over GF(2) with the reference's pivot rule (first candidate row):
    returns (L dense bool, U dense bool, chosen_pivots, invertible)."""
    n = X.shape[0]
    Y1 = np.eye(n, dtype=bool)
    Y2 = (np.asarray(X) != 0)
    piv = np.zeros(n, dtype=np.int64)
    used = np.zeros(n, dtype=bool)
    for col in range(n):
        cand = np.nonzero(Y2[:, col] & ~used)[0]
        if cand.size == 0:
            return Y1, Y2, np.zeros(n, dtype=np.int64), False
        p = cand[0]
        piv[col] = p
        used[p] = True
        others = cand[1:]
        if others.size:
            Y2[others] ^= Y2[p]
            Y1[others, p] = True
    return Y1, Y2, piv, True


class EncoderPlan:
    """The encoding structure the reference derives from H (row-oriented CSR pieces)."""

    def __init__(self, H):
        H = sp.csr_matrix(H)
        M, N = H.shape
        K = N - M
        self.N, self.K, self.M = N, K, M
        last = sp.csr_matrix(H[:, K:])
        shape = _is_full_diag_triangular(last)
        self.row_order = None
        self.L = None
        if shape != 0:
            self.algo = "Forward Substitution" if shape == 1 else "Backward Substitution"
            P = sp.tril(last, -1) if shape == 1 else sp.triu(last, 1)
            self.direction = 1 if shape == 1 else -1
        else:
            rev = last[::-1, :]
            rshape = _is_full_diag_triangular(rev)
            if rshape != 0:
                self.algo = "Forward Substitution" if rshape == 1 else "Backward Substitution"
                self.row_order = np.arange(M)[::-1].copy()
                P = sp.tril(rev, -1) if rshape == 1 else sp.triu(rev, 1)
                self.direction = 1 if rshape == 1 else -1
            else:
                self.algo = "Matrix Inverse"
                L, U, piv, ok = gf2factorize(last.toarray())
                if not ok:
                    raise ValueError("the last N-K columns of H are singular in GF(2): not encodable")
                self.L = sp.csr_matrix(np.tril(L, -1).astype(np.int8))
                self.row_order = piv
                P = sp.triu(sp.csr_matrix(U[piv, :].astype(np.int8)), 1)
                self.direction = -1
        self.A = sp.csr_matrix(H[:, :K])
        self.P = sp.csr_matrix(P)


def _subst(r: np.ndarray, T: sp.csr_matrix, direction: int) -> np.ndarray:
    v = r.copy()
    rows = range(v.shape[0]) if direction > 0 else range(v.shape[0] - 1, -1, -1)
    ip, ix = T.indptr, T.indices
    for i in rows:
        js = ix[ip[i]:ip[i + 1]]
        if js.size:
            v[i] ^= np.bitwise_xor.reduce(v[js], axis=0)
    return v


def encode(plan: EncoderPlan, X: np.ndarray) -> np.ndarray:
    """[K] or [K][B] information bits -> [N] / [N][B] systematic codewords (uint8)."""
    X = np.asarray(X, dtype=np.uint8)
    one = X.ndim == 1
    if one:
        X = X[:, None]
    r = (plan.A.astype(np.int64) @ X.astype(np.int64)) & 1
    r = r.astype(np.uint8)
    if plan.L is not None:
        r = _subst(r, plan.L, 1)
    if plan.row_order is not None:
        r = r[plan.row_order]
    p = _subst(r, plan.P, plan.direction)
    Y = np.vstack([X, p])
    return Y[:, 0] if one else Y
