"""NumPy restatement of the reference's CPU decode path ``decode_on_host``.  TEST INFRASTRUCTURE
AND CPU BASELINE ONLY.

Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg import this module: it is the reference's
own CPU decoder (BASELINE config C1) restated so that it can run on the GPU box, where the reference
itself never travels. The product package never imports it.

What it restates, operation for operation (one codeword per call, ``imax`` iterations, no early
stop, no matching — the host path has none):

* regular class ``Discrete_LDPC_Decoder_class.decode_on_host``
  (``Discrete_LDPC_decoding/discrete_LDPC_decoder.py:357-400``): the channel value of every variable
  is scattered to its check-node inbox slots (:361-367); then for ``iter`` in ``0..imax-1`` one
  check pass (``discrete_cn_operation`` :302-335 over every check's "all but one" input rows) and
  one variable pass (``discrete_vn_operation`` :337-355, channel first); the decision is the
  variable fold over the channel and ALL inputs with the tables of ``imax-1`` (:396-398). (The last
  variable pass feeds nothing — the reference runs it anyway, and so does this restatement.)
* irregular class ``Discrete_LDPC_Decoder_class_irregular.decode_on_host``
  (``discrete_LDPC_decoder_irreg.py:439-517``): per degree group; check pass 0, then ``imax-1``
  rounds of {variable pass ``iter``, check pass ``iter+1``}, then the decision (:507-517); table
  offsets use ``d_c_max`` / ``d_v_max`` (:380-383, :411-412).

Each pass is the reference's numpy shape of work: a gather of every node's inbox rows
(``all_messages``), a gather of the d(d-1) "others" entries (``reduced``), the d-1 (or d-2) chained
table lookups on the whole [rows] vector, and a scatter to the other inbox. By default the "others"
index pattern (built in the reference from ``np.kron`` / ``np.eye`` masks every pass) is built once per
degree and the inboxes are flat vectors (shape-optimised); ``faithful_shape=True`` keeps the
reference's shape of work as well: the masks rebuilt with ``np.kron`` / ``np.eye`` in every pass
(``discrete_LDPC_decoder.py:376-378,385-388``, ``discrete_LDPC_decoder_irreg.py:462-465,482-485,498-501``),
the channel matrix built with ``np.kron`` (:361), and [E][1] inboxes addressed through column 0. Both
give identical outputs; the bench reports both per-core rates.
Pinned: equal, bit for bit, to the reference's own outputs in ``tests/golden/reference_host.npz``
(``tests/test_cpu_oracle.py``).
"""
from __future__ import annotations

import numpy as np

__all__ = ["HostDecoder"]


def _others(d: int) -> np.ndarray:
    """Column pattern of the d(d-1) 'all inputs but w' entries, output w major (w = 0..d-1)."""
    return np.array([j for w in range(d) for j in range(d) if j != w], dtype=np.int64)


def _others_kron(d: int) -> np.ndarray:
    """The same pattern the way the reference builds it in every pass: kron of the index column with a
    row of ones, transposed, masked by the off-diagonal of eye(d)."""
    m = np.kron(np.arange(d)[:, np.newaxis], np.ones(d))
    return m.transpose()[(1 - np.eye(d)).astype(bool)].astype(int)


class HostDecoder:
    """decode_on_host for one code and one table set. ``regular`` selects the regular class's
    schedule and table offsets (degrees from the first node, as ``degree_*_nr[0]`` there)."""

    def __init__(self, g, Tc: int, T: int, imax: int, cn_lut, vn_lut, regular: bool, faithful_shape: bool = False):
        self.g, self.Tc, self.T, self.imax, self.regular = g, int(Tc), int(T), int(imax), bool(regular)
        self.faithful = bool(faithful_shape)
        self.cn_lut = np.asarray(cn_lut, dtype=np.int64)
        self.vn_lut = np.asarray(vn_lut, dtype=np.int64)
        cdeg, vdeg = np.asarray(g.cn_deg), np.asarray(g.vn_deg)
        self.CM = int(cdeg[0]) if regular else int(cdeg.max())
        self.VM = int(vdeg[0]) if regular else int(vdeg.max())
        if cdeg.min() < 3 or vdeg.min() < 2:
            # degree-2 checks index a missing column, degree-1 variables reshape to (-1, 0) (App. C2)
            raise ValueError("the reference host path needs check degrees >= 3 and variable degrees >= 2")
        self.checks = []     # per degree: (rows [n, d] of CN-order edges, "others" pattern, targets)
        for d in np.unique(cdeg):
            st = np.asarray(g.cn_start)[cdeg == d]
            rows = st[:, None] + np.arange(d)
            self.checks.append((int(d), rows, _others(int(d)), np.asarray(g.tgt_cn)[rows].reshape(-1)))
        self.vars = []       # per degree: (node mask, rows [n, d] of VN-order edges, pattern, targets)
        for d in np.unique(vdeg):
            sel = vdeg == d
            st = np.asarray(g.vn_start)[sel]
            rows = st[:, None] + np.arange(d)
            self.vars.append((int(d), sel, rows, _others(int(d)), np.asarray(g.tgt_vn)[rows].reshape(-1)))

    # discrete_cn_operation (:302-335 regular, :351-407 irregular): y = [rows][d-1] others
    def _cn_op(self, y: np.ndarray, it: int) -> np.ndarray:
        Tc, T, L = self.Tc, self.T, self.cn_lut
        d = y.shape[1] + 1
        if it == 0:
            t = L[y[:, 0] * Tc + y[:, 1]]
            for l in range(d - 3):
                t = L[t * T + y[:, l + 2] + Tc * Tc + l * T * Tc]
            return t
        base = (self.CM - 3) * Tc * T + Tc * Tc + (it - 1) * (self.CM - 2) * T * T
        t = L[y[:, 0] * T + y[:, 1] + base]
        for l in range(d - 3):
            t = L[t * T + y[:, l + 2] + (l + 1) * T * T + base]
        return t

    # discrete_vn_operation (:337-355 / :409-437): y = [rows][k], column 0 the channel value
    def _vn_op(self, y: np.ndarray, it: int) -> np.ndarray:
        Tc, T, L = self.Tc, self.T, self.vn_lut
        base = (Tc * T + (self.VM - 1) * T * T) * it
        t = L[y[:, 0] * T + y[:, 1] + base]
        for l in range(y.shape[1] - 2):
            t = L[t * T + y[:, l + 2] + l * T * T + base + Tc * T]
        return t

    def _check_pass(self, cin: np.ndarray, vin: np.ndarray, it: int) -> None:
        for d, rows, oth, tgt in self.checks:
            if self.faithful:                                  # [E][1] inboxes, masks rebuilt every pass
                red = cin[rows][:, _others_kron(d)].reshape(-1, d - 1)
                vin[tgt, 0] = self._cn_op(red, it)
                continue
            allm = cin[rows]                                   # all_messages
            red = allm[:, oth].reshape(-1, d - 1)              # reduced: one row per output edge
            vin[tgt] = self._cn_op(red, it)

    def _var_pass(self, ch: np.ndarray, vin: np.ndarray, cin: np.ndarray, it: int) -> None:
        for d, sel, rows, oth, tgt in self.vars:
            if self.faithful:
                chm = np.kron(ch[sel][:, np.newaxis], np.ones((d, 1))).astype(int)
                red = vin[rows][:, _others_kron(d)].reshape(-1, d - 1)
                cin[:, 0][tgt] = self._vn_op(np.hstack((chm, red)), it)
                continue
            chm = np.repeat(ch[sel], d)[:, None]               # channel_val_mat (np.kron of the column)
            red = vin[rows][:, oth].reshape(-1, d - 1)
            cin[tgt] = self._vn_op(np.hstack((chm, red)), it)

    def decode(self, channel_values: np.ndarray) -> np.ndarray:
        """One codeword: [N] channel cluster ids -> [N] decided cluster ids (int64)."""
        g = self.g
        ch = np.asarray(channel_values).astype(np.int64).reshape(-1)
        shape = (g.n_e, 1) if self.faithful else (g.n_e,)
        cin = np.zeros(shape, dtype=np.int64)
        vin = np.zeros(shape, dtype=np.int64)
        for d, sel, rows, _, tgt in self.vars:                 # send the channel values
            if self.faithful:
                cin[:, 0][tgt] = np.kron(ch[sel][:, np.newaxis], np.ones((d, 1))).astype(int).reshape(-1)
            else:
                cin[tgt] = np.repeat(ch[sel], d)
        if self.regular:
            for it in range(self.imax):
                self._check_pass(cin, vin, it)
                self._var_pass(ch, vin, cin, it)
        else:
            self._check_pass(cin, vin, 0)
            for it in range(self.imax - 1):
                self._var_pass(ch, vin, cin, it)
                self._check_pass(cin, vin, it + 1)
        out = np.zeros(g.n_v, dtype=np.int64)
        for d, sel, rows, _, _ in self.vars:                   # decision over all inputs
            allm = vin[rows][:, :, 0] if self.faithful else vin[rows]
            out[sel] = self._vn_op(np.hstack((ch[sel][:, None], allm)), self.imax - 1)
        return out
