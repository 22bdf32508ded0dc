"""Irregular information-bottleneck LDPC decoder — drop-in for the reference's
``Discrete_LDPC_decoding/discrete_LDPC_decoder_irreg.py`` (class
``Discrete_LDPC_Decoder_class_irregular``, :22-517), running on MI355X HIP kernels.

Same constructor, attributes and methods; ``decode_OpenCL`` / ``return_errors_all_zero`` /
``decode_on_host`` execute ``libibldpc.so`` (``ibl_ib_decode``, ``ibl_count_below``).
"""
from __future__ import annotations

import numpy as np
import torch

from ._dropin import CodeMixin, is_true, resolve_device, to_device_input
from .engine import IBDecoder, count_below
from .tables import IBTables, identity_matching


class Discrete_LDPC_Decoder_class_irregular(CodeMixin):
    """Reference ``__init__`` (discrete_LDPC_decoder_irreg.py:34-67)."""

    def __init__(self, filename, imax_, cardinality_T_channel_, cardinality_T_decoder_ops_,
                 Trellis_checknode_vector_a_, Trellis_varnode_vector_a_, matching_vector_checknode_,
                 matching_vector_varnode_, msg_at_time_, match='true'):
        self._init_code(filename)
        self.imax = int(imax_)
        self.cardinality_T_channel = int(cardinality_T_channel_)
        self.cardinality_T_decoder_ops = int(cardinality_T_decoder_ops_)
        self.Trellis_checknode_vector_a = np.asarray(Trellis_checknode_vector_a_).astype(int)
        self.Trellis_varnode_vector_a = np.asarray(Trellis_varnode_vector_a_).astype(int)
        self.set_code_parameters()
        self.data_len = int(self.R_c * self.codeword_len)   # reference :59 (float R_c)
        self.msg_at_time = int(msg_at_time_)
        self.map_node_connections()
        self.matching_vector_checknode = matching_vector_checknode_
        self.matching_vector_varnode = matching_vector_varnode_
        self.match = match
        self._dec = None
        self._host_dec = None
        self.device = None

    # -- tables -----------------------------------------------------------------
    def _tables(self) -> IBTables:
        T, Tc = self.cardinality_T_decoder_ops, self.cardinality_T_channel
        mc = self.matching_vector_checknode
        mv = self.matching_vector_varnode
        mc = identity_matching(T, self.d_c_max, self.imax) if mc is None else np.asarray(mc).ravel()
        mv = identity_matching(T, self.d_v_max, self.imax) if mv is None else np.asarray(mv).ravel()
        return IBTables(Tc, T, self.d_c_max, self.d_v_max, self.imax,
                        np.asarray(self.Trellis_checknode_vector_a, np.int32).ravel(),
                        np.asarray(self.Trellis_varnode_vector_a, np.int32).ravel(),
                        mc.astype(np.int32), mv.astype(np.int32))

    def update_trellis_vectors(self, Trellis_checknode_vector_a_, Trellis_varnode_vector_a_):
        self.Trellis_checknode_vector_a = np.asarray(Trellis_checknode_vector_a_).astype(int)
        self.Trellis_varnode_vector_a = np.asarray(Trellis_varnode_vector_a_).astype(int)
        self._dec = self._host_dec = None
        if self.device is not None:
            self.init_OpenCL_decoding(self.msg_at_time, self.device)

    # -- reference API ----------------------------------------------------------------
    def init_OpenCL_decoding(self, msg_at_time_, context_=False):
        """Upload graph + tables to the device and size the inboxes (reference :172-243)."""
        dev = resolve_device(context_)
        self.device = dev
        self.context = dev
        self.msg_at_time = int(msg_at_time_)
        self._dec = IBDecoder(self._graph_on(dev), self._tables(), is_true(self.match), self.msg_at_time)

    def decode_OpenCL(self, received_blocks, buffer_in=False, return_buffer=False, out_dtype=torch.int32):
        """Decode [N][B] channel cluster ids (reference :245-341); batch-global early stop."""
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
        """Number of decided 1-bits (cluster < T/2) in the first data_len rows (reference :343-349)."""
        buf = varnode_output_buffer
        if not isinstance(buf, torch.Tensor):
            buf = torch.from_numpy(np.ascontiguousarray(buf, dtype=np.int32)).to(self.device)
        return int(count_below(buf.contiguous(), self.data_len, self.cardinality_T_decoder_ops // 2).item())

    def decode_on_host(self, channel_values_):
        """One codeword, exactly imax iterations, no matching — the semantics of the reference's
        CPU path (:439-517), executed by the same HIP kernels (no CPU decoder exists here)."""
        if self.device is None:
            self.init_OpenCL_decoding(self.msg_at_time)
        if self._host_dec is None:
            self._host_dec = IBDecoder(self._graph_on(self.device), self._tables(), False, 1)
        ch = torch.from_numpy(np.asarray(channel_values_, dtype=np.int32).reshape(-1, 1).copy()).to(self.device)
        out = self._host_dec.decode(ch, out_dtype=torch.int32, early_stop=False)
        return out[:, 0].cpu().numpy().astype(np.float64)
