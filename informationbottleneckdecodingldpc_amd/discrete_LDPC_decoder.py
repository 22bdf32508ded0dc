"""Regular information-bottleneck LDPC decoder — drop-in for the reference's
``Discrete_LDPC_decoding/discrete_LDPC_decoder.py`` (class ``Discrete_LDPC_Decoder_class``,
:19-400), running on MI355X HIP kernels.

The regular kernels (``kernels_template.cl``) are the irregular ones with one degree per node
type and no matching; the same ``ibl_ib`` engine serves both (the LUT offsets coincide because
``d_c_max``/``d_v_max`` equal the node degrees).
"""
from __future__ import annotations

import numpy as np
import torch

from ._dropin import CodeMixin, resolve_device, to_device_input
from .engine import IBDecoder, count_below
from .tables import IBTables, identity_matching


class Discrete_LDPC_Decoder_class(CodeMixin):
    """Reference ``__init__`` (discrete_LDPC_decoder.py:30-51)."""

    def __init__(self, filename, imax_, cardinality_T_channel_, cardinality_T_decoder_ops_,
                 Trellis_checknode_vector_a_, Trellis_varnode_vector_a_, msg_at_time_):
        self._init_code(filename)
        self.imax = int(imax_)
        self.cardinality_T_channel = int(cardinality_T_channel_)
        self.cardinality_T_decoder_ops = int(cardinality_T_decoder_ops_)
        self.Trellis_checknode_vector_a = np.asarray(Trellis_checknode_vector_a_).astype(int)
        self.Trellis_varnode_vector_a = np.asarray(Trellis_varnode_vector_a_).astype(int)
        self.msg_at_time = int(msg_at_time_)
        self.map_node_connections()
        self.R_c = self.edges.R_c
        self.data_len = self.edges.data_len
        self._dec = None
        self.device = None

    def _tables(self) -> IBTables:
        T, Tc = self.cardinality_T_decoder_ops, self.cardinality_T_channel
        return IBTables(Tc, T, self.d_c_max, self.d_v_max, self.imax,
                        np.asarray(self.Trellis_checknode_vector_a, np.int32).ravel(),
                        np.asarray(self.Trellis_varnode_vector_a, np.int32).ravel(),
                        identity_matching(T, self.d_c_max, self.imax), identity_matching(T, self.d_v_max, self.imax))

    def update_trellis_vectors(self, Trellis_checknode_vector_a_, Trellis_varnode_vector_a_):
        """Reference :53-55."""
        self.Trellis_checknode_vector_a = np.asarray(Trellis_checknode_vector_a_).astype(int)
        self.Trellis_varnode_vector_a = np.asarray(Trellis_varnode_vector_a_).astype(int)
        self._dec = None
        if self.device is not None:
            self.init_OpenCL_decoding(self.msg_at_time, self.device)

    def init_OpenCL_decoding(self, msg_at_time_, context_=False):
        """Reference :132-200."""
        dev = resolve_device(context_)
        self.device = dev
        self.context = dev
        self.msg_at_time = int(msg_at_time_)
        self._dec = IBDecoder(self._graph_on(dev), self._tables(), False, self.msg_at_time)

    def decode_OpenCL(self, received_blocks, buffer_in=False, return_buffer=False, out_dtype=torch.int32):
        """Reference :202-295."""
        if self._dec is None:
            self.init_OpenCL_decoding(self.msg_at_time)
        ch = to_device_input(received_blocks, buffer_in, self.device, (torch.int32, torch.uint8))
        if ch.shape[1] > self._dec.max_batch:
            self.init_OpenCL_decoding(ch.shape[1], self.device)
        # out_dtype: the reference's int32 cluster ids; torch.uint8 holds the same values in a quarter of the bytes
        # (the pipelined BER driver's decisions)
        out = self._dec.decode(ch, out_dtype=out_dtype, early_stop=True)
        return out if return_buffer else out.cpu().numpy()

    def return_errors_all_zero(self, varnode_output_buffer):
        """Counts decided 1-bits over ALL N rows, as the reference's regular class does (:297-300)."""
        buf = varnode_output_buffer
        if not isinstance(buf, torch.Tensor):
            buf = torch.from_numpy(np.ascontiguousarray(buf, dtype=np.int32)).to(self.device)
        return int(count_below(buf.contiguous(), buf.shape[0], self.cardinality_T_decoder_ops // 2).item())

    def decode_on_host(self, channel_values_):
        """One codeword, exactly imax iterations (reference CPU path :357-400), on the HIP kernels."""
        if self._dec is None:
            self.init_OpenCL_decoding(self.msg_at_time)
        ch = torch.from_numpy(np.asarray(channel_values_, dtype=np.int32).reshape(-1, 1).copy()).to(self.device)
        out = self._dec.decode(ch, out_dtype=torch.int32, early_stop=False)
        return out[:, 0].cpu().numpy()
