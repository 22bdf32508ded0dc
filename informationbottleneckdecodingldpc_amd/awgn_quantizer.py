"""Drop-in for ``AWGN_Channel_Transmission/AWGN_Quantizer_BPSK.py`` ``AWGN_Channel_Quantizer`` —
the channel side of the BER drivers (``DVB-S2/BER_simulation_OpenCL.py:94-111``).

Same constructor, attribute names and methods. Differences a caller can see:

* the quantiser DESIGN (``calc_quanti``, :62-97) runs the information-bottleneck package
  ``ib_base``, which is not part of the reference repository; here ``calc_quanti`` builds the
  uniform-threshold quantiser of :class:`.channel.UniformQuantizer` (same contract: ``T`` clusters
  ordered by LLR, ``cdf_t_given_x_equals_zero`` with T+1 entries, ``output_LLRs``, ``limits``).
  A designed quantiser is used by assigning its CDF / LLRs (or :meth:`from_generated`);
* ``init_OpenCL_quanti`` takes a device (index / ``torch.device``) instead of creating an OpenCL
  context, and ``context`` is that device (pass it to the decoders' ``init_OpenCL_decoding``);
* ``quantize_direct_OpenCL(_LLR)`` generate the uniforms ON the device (``ibl_channel_sample``:
  counter-based Philox, numpy-compatible stream) instead of ``np.random.rand`` + an N*B float64
  upload per batch (:231-236). Each call advances ``offset``; ``seed`` selects the stream, so a
  run is reproducible and ranks can take disjoint streams (``seed`` = base seed + rank);
* device results are torch tensors (the reference returns ``pyopencl.array``).
"""
from __future__ import annotations

import numpy as np

from .channel import UniformQuantizer

__all__ = ["AWGN_Channel_Quantizer"]


class AWGN_Channel_Quantizer:
    """Reference: ``AWGN_Quantizer_BPSK.py:24-260``."""

    def __init__(self, sigma_n2_, AD_max_abs_, cardinality_T_, cardinality_Y_, dont_calc=False, seed=0):
        self.nror = 5
        self.sigma_n2 = sigma_n2_
        self.cardinality_T = int(cardinality_T_)
        self.cardinality_Y = cardinality_Y_
        self.AD_max_abs = AD_max_abs_
        self.limits = np.zeros(self.cardinality_T)
        if cardinality_Y_ is not None and cardinality_Y_ > 1:
            self.y_vec = np.linspace(-AD_max_abs_, AD_max_abs_, cardinality_Y_)
            self.delta = self.y_vec[1] - self.y_vec[0]
        self.x_vec = np.array([-1, 1])
        self.seed = int(seed)
        self.offset = 0
        self.context = None
        if not dont_calc:
            self.calc_quanti()

    def calc_quanti(self):
        """Quantiser design (reference :62-97 runs the absent ``ib_base`` sIB): uniform thresholds."""
        q = UniformQuantizer(self.sigma_n2, T=self.cardinality_T, AD_max_abs=self.AD_max_abs)
        self.p_t_given_x_equals_zero = q.p_t_given_x0
        self.cdf_t_given_x_equals_zero = q.cdf_t_given_x_equals_zero
        self.output_LLRs = q.output_LLRs
        # limits[t] = lower border of cluster t (limits[0] = -AD_max_abs), quantize_on_host :145-154
        self.limits = np.concatenate([[-float(self.AD_max_abs)], q.limits])

    @classmethod
    def from_generated(cls, cdf_t_given_x_equals_zero_, output_LLRs_=None, seed=0):
        """A quantiser from a stored CDF (reference :99-102 passes the CDF as sigma_n2 — broken)."""
        cdf = np.asarray(cdf_t_given_x_equals_zero_, dtype=np.float64)
        q = cls(None, None, len(cdf) - 1, None, dont_calc=True, seed=seed)
        q.cdf_t_given_x_equals_zero = cdf
        if output_LLRs_ is not None:
            q.output_LLRs = np.asarray(output_LLRs_, dtype=np.float64)
        return q

    # ------------------------------------------------------------------ host paths
    def quantize_direct(self, input_bits):
        """Host direct-inversion sampling with ``np.random.rand`` (reference :126-143, same rule and
        the same uniforms for the same ``np.random`` state). The reference counts u > cdf[0] = 0 and
        subtracts 1 (-1 for u == 0) and can return T when the CDF sums to just under 1; here
        t = #{w >= 1 : u > cdf[w]} clamped to T-1, equal in every other case."""
        input_bits = np.asarray(input_bits)
        rand_u = np.random.rand(input_bits.shape[0], input_bits.shape[1])
        cdf = self.cdf_t_given_x_equals_zero
        T = self.cardinality_T
        t = (rand_u[..., None] > cdf[1:]).sum(-1)
        t = np.minimum(t, T - 1)
        mirror = input_bits.astype(bool)
        t[mirror] = T - 1 - t[mirror]
        return t if input_bits.shape[1] > 1 else t[:, 0]

    def quantize_on_host(self, x):
        """Cluster ids of received values (reference :145-154): #{t : x > limits[t]} - 1, floor 0."""
        x = np.asarray(x)
        cluster = (x[..., None] - self.limits > 0).sum(-1) - 1
        cluster[cluster == -1] = 0
        return cluster if x.ndim < 2 or x.shape[1] > 1 else cluster[:, 0]

    # ---------------------------------------------------------------- device paths
    def init_OpenCL_quanti(self, N_var, msg_at_time, return_buffer_only=False, context_=None):
        """Reference :156-179: builds the kernels and the output buffers. Here: picks the device
        (``context_``: index / ``torch.device``; default the current one) and allocates the
        [N_var][msg_at_time] cluster (int32) and LLR (float64) buffers."""
        import torch

        from .engine import _require_gpu
        dev = _require_gpu(None if context_ is None else (f"cuda:{context_}" if isinstance(context_, int) else context_))
        self.context = dev
        self.return_buffer_only = return_buffer_only
        self.N_var, self.msg_at_time = int(N_var), int(msg_at_time)
        self.cluster_buff = torch.empty((self.N_var, self.msg_at_time), dtype=torch.int32, device=dev)
        self.LLR_buff = torch.empty((self.N_var, self.msg_at_time), dtype=torch.float64, device=dev)

    def _sample(self, out, llr=None, bits=None):
        from .engine import channel_sample, philox_blocks
        channel_sample(out, self.cdf_t_given_x_equals_zero, self.seed, self.offset, llr=llr, bits=bits)
        self.offset += philox_blocks(*out.shape)
        return out

    def _buf(self, name, N_var, msg_at_time, dtype):
        import torch
        buf = getattr(self, name)
        if tuple(buf.shape) != (N_var, msg_at_time) or (dtype is not None and buf.dtype != dtype):
            buf = torch.empty((N_var, msg_at_time), dtype=dtype or buf.dtype, device=self.context)
            setattr(self, name, buf)
        return buf

    def quantize_direct_OpenCL(self, N_var, msg_at_time, dtype=None, bits=None):
        """Cluster ids of the all-zero codeword (or of ``bits``) sampled on the device
        (reference :216-240). ``dtype``: torch.int32 (reference) or torch.uint8."""
        out = self._sample(self._buf("cluster_buff", N_var, msg_at_time, dtype), bits=bits)
        return out if self.return_buffer_only else out.cpu().numpy()

    def quantize_direct_OpenCL_LLR(self, N_var, msg_at_time, dtype=None, bits=None):
        """LLRs ``output_LLRs[t]`` of device-sampled clusters (reference :242-260).
        ``dtype``: torch.float64 (reference) or torch.float32."""
        out = self._sample(self._buf("LLR_buff", N_var, msg_at_time, dtype), llr=self.output_LLRs, bits=bits)
        return out if self.return_buffer_only else out.cpu().numpy()
