"""BER simulation driver — the Eb/N0 state machine of the reference's drivers
(``Irregular_LDPC_Decoding/DVB-S2/BER_simulation_OpenCL.py:76-173``, min-sum / BP variants
``BER_simulation_OpenCL_min_sum.py``, ``WLAN/BER_simulation_OpenCL_quant_BP.py:62-188``) over the
drop-in decoder classes and the device channel generator.

Per Eb/N0 point: sigma_n^2 = 10^(-Eb/N0/10) / (2 R_c) (:92); a quantiser for that noise level;
``decoder.init_OpenCL_decoding(msg_at_time, quanti.context)``; batches of ``msg_at_time``
all-zero codewords sampled ON the device, decoded, and their decided 1-bits counted
(``return_errors_all_zero``) until ``min_errors`` (:105-112); BER = errors / (R_c * blocks * N)
(:136). Next point: + small step if BER < ``BER_go_on_in_smaller_steps`` else + normal step, while
BER > ``target_error_rate`` and Eb/N0 < ``EbN0_dB_max_value`` (:156-163). Results are saved as the
reference's ``BER_results.npz`` keys (``EbN0_dB_vector``, ``BER_vector``).

Multi-GPU: one process per GPU (torch.distributed initialised by the caller); rank r draws its
channel from Philox key ``seed + r`` (disjoint streams), and the error / block counters are summed
over ranks (one small all-reduce per ``sync_every`` batches) so every rank stops at the same point.
``max_blocks`` bounds a point (the reference loops until ``min_errors`` however long that takes).

``encoded=True`` transmits random encoded codewords instead (the reference's
``LDPC_BPSK_Transmitter`` + encoder path, AWGN_Channel_Transmission/LDPC_Transmitter.py:109-125): bits
from the device Philox stream (key ``(seed + rank, 1)``, disjoint from the channel's ``(seed + rank, 0)``),
batched device encoding, the channel mirrored by
the codeword bits, and decided bits compared with the transmitted ones (``ibl_count_errors``) over the
rows ``return_errors_all_zero`` counts.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np

__all__ = ["BERConfig", "BERResult", "run_ber", "decoder_kind"]


@dataclass
class BERConfig:
    EbN0_dB_start: float = 0.0
    EbN0_dB_max_value: float = 1.2
    target_error_rate: float = 1e-6
    BER_go_on_in_smaller_steps: float = 1e-5
    EbN0_dB_normal_stepwidth: float = 0.1
    EbN0_dB_small_stepwidth: float = 0.05
    min_errors: int = 5000
    msg_at_time: int = 2
    AD_max_abs: float = 3.0
    cardinality_Y_channel: int = 2000
    cardinality_T_channel: int = 16
    max_blocks: Optional[int] = None      # per point, summed over ranks; None = until min_errors
    seed: int = 0
    sync_every: int = 1                   # batches between cross-rank counter reductions
    llr_dtype: Optional[object] = None    # float decoders: torch dtype of the channel LLRs
    encoded: bool = False                 # random encoded codewords (LDPC_BPSK_Transmitter) instead of all-zero


@dataclass
class BERResult:
    EbN0_dB_vector: np.ndarray
    BER_vector: np.ndarray
    errors: List[int] = field(default_factory=list)
    blocks: List[int] = field(default_factory=list)
    seconds: List[float] = field(default_factory=list)

    def save(self, pathname: str) -> str:
        os.makedirs(pathname, exist_ok=True)
        path = os.path.join(pathname, "BER_results.npz")
        np.savez(path, EbN0_dB_vector=self.EbN0_dB_vector, BER_vector=self.BER_vector,
                 errors=np.asarray(self.errors), blocks=np.asarray(self.blocks), seconds=np.asarray(self.seconds))
        return path


def decoder_kind(decoder) -> str:
    """'ib' (cluster-id input, ``decode_OpenCL``), 'minsum' or 'bp' (LLR input)."""
    if hasattr(decoder, "decode_OpenCL_belief_propagation") and type(decoder).__name__.startswith("Belief"):
        return "bp"
    if hasattr(decoder, "decode_OpenCL_min_sum") and type(decoder).__name__.startswith("Min_Sum"):
        return "minsum"
    if hasattr(decoder, "decode_OpenCL"):
        return "ib"
    raise TypeError(f"not a decoder class: {type(decoder).__name__}")


def _allreduce(vals):
    try:
        import torch
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return vals
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return vals
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return [float(x) for x in t.cpu().tolist()]


def _rank() -> int:
    try:
        import torch.distributed as dist
        return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    except ImportError:  # pragma: no cover
        return 0


def run_ber(decoder, cfg: BERConfig, quantizer_factory: Optional[Callable] = None,
            log: Optional[Callable[[str], None]] = None) -> BERResult:
    """Run the Eb/N0 sweep with ``decoder`` (a drop-in decoder instance). ``quantizer_factory(sigma_n2)``
    returns a quantiser object with the reference methods (default: :class:`.awgn_quantizer.AWGN_Channel_Quantizer`
    with ``cfg.cardinality_T_channel`` clusters)."""
    from .awgn_quantizer import AWGN_Channel_Quantizer
    kind = decoder_kind(decoder)
    N_var = int(decoder.codeword_len)
    R_c = float(decoder.R_c)
    rank = _rank()
    if quantizer_factory is None:
        def quantizer_factory(s2):
            return AWGN_Channel_Quantizer(s2, cfg.AD_max_abs, cfg.cardinality_T_channel, cfg.cardinality_Y_channel)
    ebn0 = [float(cfg.EbN0_dB_start)]
    ber: List[float] = [0.0]
    res = BERResult(np.array([]), np.array([]))
    offset = 0
    tx = None
    if cfg.encoded:
        import torch
        from .engine import count_errors
        from .ldpc_encoder import LDPC_BPSK_Transmitter
        tx = LDPC_BPSK_Transmitter(decoder.H_sparse, cfg.msg_at_time, seed=int(cfg.seed) + rank,
                                   device=getattr(decoder, "device", None))
        # rows return_errors_all_zero counts: all N for the regular IB class (:297-300), data_len otherwise
        err_rows = N_var if type(decoder).__name__ == "Discrete_LDPC_Decoder_class" else int(decoder.data_len)
        thr = decoder.cardinality_T_decoder_ops // 2 if kind == "ib" else 0.0
        cnt = torch.zeros(1, dtype=torch.int64, device=tx.encoder.device)
    while True:
        EbN0_dB = ebn0[-1]
        sigma_n2 = 10 ** (-EbN0_dB / 10) / (2 * R_c)
        quanti = quantizer_factory(sigma_n2)
        quanti.seed = int(cfg.seed) + rank
        quanti.offset = offset
        quanti.init_OpenCL_quanti(N_var, cfg.msg_at_time, return_buffer_only=True,
                                  context_=getattr(decoder, "device", None))
        decoder.init_OpenCL_decoding(cfg.msg_at_time, quanti.context)
        errors = 0.0
        blocks = 0
        pend_err = pend_blk = 0
        nb = 0
        t0 = time.time()
        while errors < cfg.min_errors and (cfg.max_blocks is None or blocks < cfg.max_blocks):
            kw = {} if tx is None else {"bits": tx.transmit_bits()}
            if kind == "ib":
                rec = quanti.quantize_direct_OpenCL(N_var, cfg.msg_at_time, **kw)
                dec = decoder.decode_OpenCL(rec, buffer_in=True, return_buffer=True)
            else:
                rec = quanti.quantize_direct_OpenCL_LLR(N_var, cfg.msg_at_time, dtype=cfg.llr_dtype, **kw)
                fn = decoder.decode_OpenCL_min_sum if kind == "minsum" else decoder.decode_OpenCL_belief_propagation
                dec = fn(rec, buffer_in=True, return_buffer=True)
            if tx is None:
                pend_err += decoder.return_errors_all_zero(dec)
            else:
                pend_err += int(count_errors(dec.contiguous(), err_rows, thr, kw["bits"], cnt).item())
            pend_blk += cfg.msg_at_time
            nb += 1
            if nb % max(1, cfg.sync_every) == 0:
                e, b = _allreduce([pend_err, pend_blk])
                errors += e              # integer counts, summed exactly in float64
                blocks += int(round(b))
                pend_err = pend_blk = 0
        if pend_blk:
            e, b = _allreduce([pend_err, pend_blk])
            errors += e
            blocks += int(round(b))
        offset = quanti.offset
        spent = time.time() - t0
        ber[-1] = errors / (R_c * blocks * N_var) if blocks else 0.0
        res.errors.append(errors)
        res.blocks.append(blocks)
        res.seconds.append(spent)
        if log:
            log(f"EbN0_dB={EbN0_dB:.3f} BER={ber[-1]:.3e} errors={errors:.0f} blocks={blocks} "
                f"bitrate={R_c * blocks * N_var / max(spent, 1e-9):.3e} bit/s")
        if ber[-1] > cfg.target_error_rate and EbN0_dB < cfg.EbN0_dB_max_value:
            step = cfg.EbN0_dB_small_stepwidth if ber[-1] < cfg.BER_go_on_in_smaller_steps \
                else cfg.EbN0_dB_normal_stepwidth
            ebn0.append(ebn0[-1] + step)
            ber.append(0.0)
        else:
            break
    res.EbN0_dB_vector = np.asarray(ebn0)
    res.BER_vector = np.asarray(ber)
    return res
