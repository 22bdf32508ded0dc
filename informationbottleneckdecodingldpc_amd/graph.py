"""Edge-index arrays of the Tanner graph (reference ``map_node_connections``).

Two edge orderings, exactly as the reference's inboxes
(``Discrete_LDPC_decoding/discrete_LDPC_decoder_irreg.py:121-170``,
regular copy ``discrete_LDPC_decoder.py:88-130``):

* **CN order** (CSR edge id): check-major, ascending column. ``checknode_inbox`` rows
  (variable→check messages) are indexed by it. ``cn_start`` = CSR ``indptr[:-1]``
  (``inbox_memory_start_checknodes``).
* **VN order** (CSC edge id): variable-major, ascending row. ``varnode_inbox`` rows
  (check→variable messages) are indexed by it. ``vn_start`` = CSC ``indptr[:-1]``
  (``inbox_memory_start_varnodes``).

``tgt_cn[csr_e]`` is the VN-order position of the same edge
(``target_memory_cells_checknodes``, where a check writes its output for that edge);
``tgt_vn[csc_e]`` the CN-order position (``target_memory_cells_varnodes``). They are
inverse permutations of each other.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp

from .codes import canonical_csr, code_rate

__all__ = ["EdgeGraph", "build_graph"]


@dataclass
class EdgeGraph:
    n_v: int                 # variable nodes (codeword length N)
    n_c: int                 # check nodes M
    n_e: int                 # edges E
    csr_indptr: np.ndarray   # int32 [M+1]
    csr_cols: np.ndarray     # int32 [E]   (customers_checknode_nr)
    csc_indptr: np.ndarray   # int32 [N+1]
    csc_rows: np.ndarray     # int32 [E]   (customers_varnode_nr)
    cn_deg: np.ndarray       # int32 [M]   degree_checknode_nr
    vn_deg: np.ndarray       # int32 [N]   degree_varnode_nr
    cn_start: np.ndarray     # int32 [M]   inbox_memory_start_checknodes
    vn_start: np.ndarray     # int32 [N]   inbox_memory_start_varnodes
    tgt_cn: np.ndarray       # int32 [E]   target_memory_cells_checknodes
    tgt_vn: np.ndarray       # int32 [E]   target_memory_cells_varnodes
    R_c: float               # reference design rate (float)
    data_len: int            # int(R_c * N)

    @property
    def d_c_max(self) -> int:
        return int(self.cn_deg.max())

    @property
    def d_v_max(self) -> int:
        return int(self.vn_deg.max())

    def to_csr(self) -> sp.csr_matrix:
        return sp.csr_matrix((np.ones(self.n_e, dtype=np.int64), self.csr_cols, self.csr_indptr),
                             shape=(self.n_c, self.n_v))


def build_graph(H) -> EdgeGraph:
    """Build every index array the decoders need from a parity-check matrix."""
    A = canonical_csr(H)
    n_c, n_v = A.shape
    E = int(A.nnz)
    if E >= 2**31 - 1:
        raise ValueError("edge count exceeds int32 indexing")
    indptr = A.indptr.astype(np.int64)
    cols = A.indices.astype(np.int64)
    rows = np.repeat(np.arange(n_c, dtype=np.int64), np.diff(indptr))
    # CSR edge ids sorted by (col, row) give CSC order: position p holds csr edge order[p]
    order = np.lexsort((rows, cols))
    tgt_vn = order.astype(np.int32)                 # csc position -> csr edge id
    tgt_cn = np.empty(E, dtype=np.int32)
    tgt_cn[order] = np.arange(E, dtype=np.int32)    # csr edge id -> csc position
    vn_deg = np.bincount(cols, minlength=n_v).astype(np.int32)
    cn_deg = np.diff(indptr).astype(np.int32)
    csc_indptr = np.zeros(n_v + 1, dtype=np.int64)
    np.cumsum(vn_deg, out=csc_indptr[1:])
    R_c = float(code_rate(A))
    return EdgeGraph(
        n_v=int(n_v), n_c=int(n_c), n_e=E,
        csr_indptr=indptr.astype(np.int32), csr_cols=cols.astype(np.int32),
        csc_indptr=csc_indptr.astype(np.int32), csc_rows=rows[order].astype(np.int32),
        cn_deg=cn_deg, vn_deg=vn_deg,
        cn_start=indptr[:-1].astype(np.int32), vn_start=csc_indptr[:-1].astype(np.int32),
        tgt_cn=tgt_cn, tgt_vn=tgt_vn,
        R_c=R_c, data_len=int(R_c * n_v),
    )
