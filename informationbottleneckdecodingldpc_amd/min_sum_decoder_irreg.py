"""Float min-sum LDPC decoder — drop-in for the reference's
``Continous_LDPC_Decoding/min_sum_decoder_irreg.py`` (class ``Min_Sum_Decoder_class_irregular``,
:19-385), running on MI355X HIP kernels (``ibl_float_*``).

``precision`` (extension, keyword-only) selects float32 (default, the BASELINE build) or
float64 (the reference's double precision, bit-identical min-sum). Output buffers carry that
dtype.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._dropin import CodeMixin, resolve_device, to_device_input
from .engine import FloatDecoder, count_below

_KIND = _lib.IBL_MINSUM


class Min_Sum_Decoder_class_irregular(CodeMixin):
    """Reference ``__init__`` (min_sum_decoder_irreg.py:23-69)."""

    _kind = _KIND

    def __init__(self, filename, imax_, cardinality_T_channel_, msg_at_time_, *, precision=torch.float32,
                 llr_max: float = 150.0):
        self._init_code(filename)
        self.imax = int(imax_)
        self.cardinality_T_channel = int(cardinality_T_channel_)
        self.set_code_parameters()
        self.data_len = int(self.R_c * self.codeword_len)
        self.msg_at_time = int(msg_at_time_)
        self.map_node_connections()
        self.precision = precision
        self.llr_max = float(llr_max)
        self._dec = None
        self.device = None

    def init_OpenCL_decoding(self, msg_at_time_, context_=False):
        """Reference :167-218."""
        dev = resolve_device(context_)
        self.device = dev
        self.context = dev
        self.msg_at_time = int(msg_at_time_)
        self._dec = FloatDecoder(self._graph_on(dev), self._kind, self.imax, self.msg_at_time,
                                 precision=self.precision, llr_max=self.llr_max)

    def _decode(self, received_blocks, buffer_in, return_buffer, early_stop=True):
        if self._dec is None:
            self.init_OpenCL_decoding(self.msg_at_time)
        llr = to_device_input(received_blocks, buffer_in, self.device, (torch.float32, torch.float64))
        if llr.shape[1] > self._dec.max_batch:
            self.init_OpenCL_decoding(llr.shape[1], self.device)
        if not return_buffer:
            # host output synchronises anyway: channel LLRs of THIS decode that break the precondition (NaN; BP:
            # also |x| > 709.78 in fp64, +-inf in fp32) raise instead of returning unspecified values
            # (FloatDecoder.input_violations); counts left by earlier return_buffer decodes are cleared first
            self._dec.input_violations(raise_on_error=False)
        out = self._dec.decode(llr, early_stop=early_stop)
        if return_buffer:
            return out
        self._dec.input_violations()
        return out.cpu().numpy()

    def decode_OpenCL_min_sum(self, received_blocks, buffer_in=False, return_buffer=False):
        """Reference :221-287."""
        return self._decode(received_blocks, buffer_in, return_buffer)

    def return_errors_all_zero(self, varnode_output_buffer):
        """Count of negative APP LLRs in the first data_len rows, as a float (reference :290-295)."""
        buf = varnode_output_buffer
        if not isinstance(buf, torch.Tensor):
            buf = torch.from_numpy(np.ascontiguousarray(buf, dtype=np.float64)).to(self.device)
        return float(count_below(buf.contiguous(), self.data_len, 0.0).item())

    def decode_on_host(self, channel_values_):
        """One codeword, exactly imax iterations, the kernels' semantics (the reference's CPU path is
        broken) — executed on the GPU."""
        out = self._decode(np.asarray(channel_values_, dtype=np.float64).reshape(-1, 1), False, True,
                           early_stop=False)
        return out[:, 0].double().cpu().numpy()
