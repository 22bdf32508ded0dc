"""Drop-in for the reference's systematic LDPC encoder (``Discrete_LDPC_decoding/LDPC_encoder.py``)
and its BPSK transmitter (``AWGN_Channel_Transmission/LDPC_Transmitter.py``), batched on the device.

``LDPCEncoder(filename)`` derives the same encoding plan as ``getLDPCEncoderParamters`` (:197-269)
— natively, inside ``ibl_encoder_create`` — and exposes the reference's attributes
(``N``, ``K``, ``NumInfoBits``, ``NumParityBits``, ``BlockLength``, ``EncodingAlgorithm``).
``encode`` / ``encode_c`` (:86-162) take one information word like the reference; ``encode_batch``
takes a u8 [K][B] device tensor and encodes all B words in one call (the reference loops over
``msg_at_time`` columns, LDPC_Transmitter.py:116-117). Encoding runs only in ``libibldpc.so``.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import codes
from ._dropin import load_H, resolve_device
from .engine import Encoder, philox_blocks, random_bits

__all__ = ["LDPCEncoder", "LDPC_BPSK_Transmitter"]


class LDPCEncoder:
    """Systematic encoder of H = [A | B]: codeword = [x; p] with H [x; p] = 0 over GF(2)."""

    def __init__(self, filename, alist_file: bool = True, max_batch: int = 1, device=None):
        self.H_sparse = load_H(filename)
        self.N = self.H_sparse.shape[1]
        self.K = self.N - self.H_sparse.shape[0]
        self.NumInfoBits = self.K
        self.NumParityBits = self.N - self.K
        self.BlockLength = self.N
        self._device = device
        self._enc: Optional[Encoder] = None
        self._ensure(max(1, int(max_batch)))
        self.EncodingAlgorithm = self._enc.algorithm

    def _ensure(self, B: int) -> Encoder:
        if self._enc is None or self._enc.max_batch < B:
            dev = resolve_device(self._device)
            cap = B if self._enc is None else max(B, 2 * self._enc.max_batch)
            self._enc = Encoder(self.H_sparse, cap, dev)
        return self._enc

    @property
    def device(self) -> torch.device:
        return self._ensure(1).device

    def encode_batch(self, info: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """u8 [K][B] device tensor -> u8 [N][B] device tensor of codewords."""
        return self._ensure(int(info.shape[1])).encode(info, out)

    def encode(self, X) -> np.ndarray:
        """One information word (length K, 0/1) -> length-N codeword (reference :86-123)."""
        X = np.asarray(X).reshape(-1)
        if X.size != self.K:
            raise ValueError(f"information word must have K={self.K} bits, got {X.size}")
        enc = self._ensure(1)
        info = torch.from_numpy((X.astype(np.int64) & 1).astype(np.uint8).reshape(-1, 1)).to(enc.device)
        return enc.encode(info)[:, 0].cpu().numpy().astype(np.int64)

    encode_c = encode   # the reference's Cython-accelerated variant (:125-162) computes the same words


class LDPC_BPSK_Transmitter:
    """Random information words, encoded and BPSK-mapped (0 -> +1, 1 -> -1), ``msg_at_time`` per call
    (LDPC_Transmitter.py:16-133). Bits come from the numpy-compatible Philox stream (key
    ``(seed, 1)`` — disjoint from the channel generator's ``(seed, 0)`` — counter ``offset``, advanced by
    each call) instead of numpy's global ``randint``.

    ``transmit()`` returns host float64 [N][msg_at_time] symbols like the reference;
    ``transmit_bits()`` keeps everything on the device and returns the u8 [N][B] codeword bits (the
    input the device channel ``quantize_direct_OpenCL(..., bits=...)`` mirrors clusters by)."""

    def __init__(self, filename_H_, msg_at_time: int = 1, seed: int = 0, device=None):
        self.filename_H = filename_H_
        self.H_sparse = load_H(filename_H_)
        self.msg_at_time = int(msg_at_time)
        self.encoder = LDPCEncoder(self.H_sparse, max_batch=self.msg_at_time, device=device)
        self.codeword_len = self.H_sparse.shape[1]
        self.N_v = self.codeword_len
        self.N_c = self.H_sparse.shape[0]
        self.R_c = codes.code_rate(self.H_sparse)
        # the reference's data_len = int(R_c * N) (:27) can be one short of K (DVB-S2: 32399 vs 32400),
        # which its encode_c call would reject; words here always have K bits
        self.data_len = int(self.R_c * self.codeword_len)
        self.K = self.encoder.K
        self.seed = int(seed)
        self.offset = 0
        self.last_transmitted_bits = []
        self._info = None
        self._code = None

    def transmit_bits(self, msg_at_time: Optional[int] = None) -> torch.Tensor:
        B = self.msg_at_time if msg_at_time is None else int(msg_at_time)
        dev = self.encoder.device
        if self._info is None or self._info.shape[1] != B:
            self._info = torch.empty((self.K, B), dtype=torch.uint8, device=dev)
            self._code = torch.empty((self.codeword_len, B), dtype=torch.uint8, device=dev)
        random_bits(self._info, self.seed, self.offset)
        self.offset += philox_blocks(self.K, B)
        self.encoder.encode_batch(self._info, self._code)
        self.last_transmitted_bits = self._info
        return self._code

    def transmit(self) -> np.ndarray:
        code = self.transmit_bits()
        self.last_transmitted_bits = self._info.cpu().numpy().astype(np.int64)
        return self.BPSK_mapping(code.cpu().numpy())

    def BPSK_mapping(self, X) -> np.ndarray:
        data = np.ones((self.codeword_len, np.asarray(X).shape[1]))
        data[np.asarray(X) == 1] = -1
        return data
