"""Shared plumbing of the reference-compatible decoder classes.

The reference classes (``Discrete_LDPC_Decoder_class[_irregular]``,
``Min_Sum_Decoder_class_irregular``, ``BeliefPropagationDecoderClassIrregular``) each carry a
copy of the same H loading and ``map_node_connections`` code; here it lives once.

Deviations kept deliberately small and documented in DESIGN.md:
* ``H`` is held as a canonical scipy CSR matrix (the reference's regular class densifies it);
* host inbox arrays (``inbox_memory_checknodes`` ...) are not allocated — the inboxes live on
  the device, sized by ``msg_at_time``;
* ``context_`` of ``init_OpenCL_decoding`` selects the HIP device: ``False``/``None`` (current
  device), an ``int`` index, a ``torch.device``, or any object with a ``.device`` attribute.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch

from . import codes
from .engine import Graph
from .graph import build_graph

def resolve_device(context_) -> torch.device:
    if context_ is False or context_ is None:
        if not torch.cuda.is_available():
            raise RuntimeError("no HIP device visible: decoding runs only on the GPU")
        return torch.device("cuda", torch.cuda.current_device())
    if isinstance(context_, int) and not isinstance(context_, bool):
        return torch.device("cuda", context_)
    if isinstance(context_, torch.device):
        return context_ if context_.index is not None else torch.device("cuda", torch.cuda.current_device())
    dev = getattr(context_, "device", None)
    if dev is not None:
        return resolve_device(dev)
    raise TypeError(f"cannot interpret context_={context_!r} as a HIP device")


def load_H(filename) -> sp.csr_matrix:
    """File name (alist / .npy / .npz) or an in-memory 0/1 matrix -> canonical CSR."""
    if isinstance(filename, (str, bytes)) or hasattr(filename, "__fspath__"):
        return codes.load_check_mat(str(filename))
    return codes.canonical_csr(filename)


class CodeMixin:
    """H analysis and the edge-index arrays (``map_node_connections``)."""

    def _init_code(self, filename):
        self.H_sparse = load_H(filename)
        self.H = self.H_sparse
        self.edges = build_graph(self.H_sparse)
        e = self.edges
        self.degree_checknode_nr = e.cn_deg.astype(np.int64)
        self.degree_varnode_nr = e.vn_deg.astype(np.int64)
        self.N_v = e.n_v
        self.N_c = e.n_c
        self.codeword_len = e.n_v
        self.d_c_max = e.d_c_max
        self.d_v_max = e.d_v_max

    def load_check_mat(self, filename):
        return load_H(filename)

    def load_sparse_csr(self, filename):
        return codes.load_check_mat(str(filename))

    def alistToNumpy(self, lines):
        return codes.alist_to_numpy(lines)

    def map_node_connections(self):
        """Edge index arrays, same names and values as the reference (see graph.py)."""
        e = self.edges
        self.inbox_memory_start_checknodes = e.cn_start.astype(np.int64)
        self.inbox_memory_start_varnodes = e.vn_start.astype(np.int64)
        self.customers_checknode_nr = e.csr_cols.astype(np.int64)
        self.customers_varnode_nr = e.csc_rows.astype(np.int64)
        self.target_memory_cells_checknodes = e.tgt_cn.astype(np.int64)
        self.target_memory_cells_varnodes = e.tgt_vn.astype(np.int64)

    def set_code_parameters(self):
        self.R_c = self.edges.R_c

    def _graph_on(self, dev: torch.device) -> Graph:
        """The device copy of the edge arrays, one per device, held by this decoder only: it is freed with
        the decoder (``Graph.__del__``), so constructing decoders per Eb/N0 point or per code does not
        accumulate device memory."""
        graphs = self.__dict__.setdefault("_device_graphs", {})
        g = graphs.get(dev.index)
        if g is None or g.edges is not self.edges:
            g = Graph(self.edges, dev)
            graphs[dev.index] = g
        return g


def to_device_input(received_blocks, buffer_in: bool, dev: torch.device, dtype) -> torch.Tensor:
    """Host ndarray (uploaded) or device tensor (``buffer_in=True``) -> contiguous [N][B] tensor."""
    if buffer_in:
        t = received_blocks
        if not isinstance(t, torch.Tensor):
            raise TypeError("buffer_in=True expects a device tensor (e.g. a quantizer's output buffer)")
        if t.device != dev:
            t = t.to(dev)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(received_blocks))).to(dev)
    if t.dim() == 1:
        t = t[:, None]
    if t.dtype not in dtype:
        t = t.to(dtype[0])
    return t.contiguous()


def is_true(match) -> bool:
    """The reference pastes ``match`` into ``#define MATCH`` ('true'/'false' strings)."""
    if isinstance(match, str):
        return match.strip().lower() in ("true", "1", "yes")
    return bool(match)
