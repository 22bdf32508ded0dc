"""BPSK/AWGN channel quantisation for the decoders' inputs (reference layer L2, host set-up).

The reference designs its channel quantiser with the information-bottleneck package
``ib_base`` (``AWGN_Channel_Transmission/AWGN_Quantizer_BPSK.py:62-97``, absent here). This module
keeps the same observable contract — ``T`` clusters ordered by LLR, cluster ``t < T/2`` meaning
bit 1, per-cluster LLRs ``log p(t|x=0)/p(t|x=1)`` (``output_LLRs``, :96) and the CDF
``p(t|x=0)`` used for direct inversion sampling (:94, ``quantize_direct`` :126-143) — with a
uniform-threshold quantiser on the received value ``y = ±1 + n`` over ``[-AD_max_abs,
AD_max_abs]``.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
from scipy.stats import norm

__all__ = ["sigma2_from_ebn0", "UniformQuantizer"]


def sigma2_from_ebn0(ebn0_db: float, R_c: float) -> float:
    """Noise variance of the reference drivers: 10^(-Eb/N0/10) / (2 R_c)
    (``Irregular_LDPC_Decoding/DVB-S2/BER_simulation_OpenCL.py:105``)."""
    return 10 ** (-ebn0_db / 10) / (2 * R_c)


@dataclass
class UniformQuantizer:
    sigma_n2: float
    T: int = 16
    AD_max_abs: float = 3.0

    def __post_init__(self):
        T = self.T
        self.limits = np.linspace(-self.AD_max_abs, self.AD_max_abs, T + 1)[1:-1]   # T-1 inner thresholds
        edges = np.concatenate([[-np.inf], self.limits, [np.inf]])
        s = np.sqrt(self.sigma_n2)
        p0 = norm.cdf((edges[1:] - 1) / s) - norm.cdf((edges[:-1] - 1) / s)   # x=0 -> +1
        p1 = norm.cdf((edges[1:] + 1) / s) - norm.cdf((edges[:-1] + 1) / s)   # x=1 -> -1
        p0 = np.maximum(p0, 1e-300)
        p1 = np.maximum(p1, 1e-300)
        self.p_t_given_x0 = p0 / p0.sum()
        self.output_LLRs = np.log(p0 / p1)
        self.cdf_t_given_x_equals_zero = np.concatenate([[0.0], np.cumsum(self.p_t_given_x0)])

    def quantize_on_host(self, y: np.ndarray) -> np.ndarray:
        """Cluster ids of received values y (ascending thresholds)."""
        return np.searchsorted(self.limits, y, side="left").astype(np.int32)

    def sample_all_zero(self, n: int, B: int, rng: np.random.Generator) -> np.ndarray:
        """[n][B] cluster ids of the all-zero codeword (BPSK +1) through the AWGN channel."""
        y = 1.0 + np.sqrt(self.sigma_n2) * rng.standard_normal((n, B))
        return self.quantize_on_host(y)

    def llr_of(self, clusters: np.ndarray) -> np.ndarray:
        return self.output_LLRs[clusters]

    # ---- device sampling (torch on the decoder's device; reference quantize_direct_OpenCL*)
    def sample_all_zero_device(self, n: int, B: int, device, generator=None, dtype=None):
        import torch
        y = torch.randn((n, B), device=device, generator=generator, dtype=torch.float32)
        y = 1.0 + float(np.sqrt(self.sigma_n2)) * y
        lim = torch.as_tensor(self.limits, dtype=torch.float32, device=device)
        t = torch.bucketize(y, lim, right=False)
        return t.to(dtype or torch.uint8).contiguous()
