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

Multi-GPU: one process per GPU (torch.distributed initialised by the caller). Batches are dealt
round-robin and every batch's channel is keyed on its GLOBAL batch index (``global_batch``), the error
counts of each round are exchanged (one small all-reduce per ``sync_every`` rounds) and walked in global
order with the reference's stop rule, so a k-rank sweep counts exactly the frames of the 1-rank sweep
(SURVEY H9). ``max_blocks`` bounds a point (the reference loops until ``min_errors`` however long that
takes).

Throughput: on a HIP device the batches of a round are pipelined — batch k+1's channel (and,
encoded, its information bits and codewords) is generated on a side stream into the other half of a double
buffer while batch k decodes on the caller's stream, batch k's error count runs on the side stream into a
device vector, and the host reads the counts once per round (``sync_every`` batches) while the next round is
already enqueued (``_DeviceRunner``). Which frames are counted does not change: the stop rule still walks the
per-batch counts in global order, so a round decoded past the stop is discarded like the rest of a round
(``cfg.pipeline=False`` runs the reference's call sequence batch by batch, ``_SyncRunner``).

``encoded=True`` transmits random encoded codewords instead (the reference's
``LDPC_BPSK_Transmitter`` + encoder path, AWGN_Channel_Transmission/LDPC_Transmitter.py:109-125): bits
from the device Philox stream (key ``(seed, 1)``, disjoint from the channel's ``(seed, 0)``; counter keyed
on the global batch index like the channel), batched device encoding, the channel mirrored by
the codeword bits, and decided bits compared with the transmitted ones (``ibl_count_errors``) over the
rows ``return_errors_all_zero`` counts.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np

__all__ = ["BERConfig", "BERResult", "run_ber", "run_ber_lockstep", "global_batch", "decoder_kind"]


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
    pipeline: bool = True                 # device double buffering + side-stream counts (see the module docstring)
    gen_chunk: int = 1 << 22              # pipelined channel: samples per side-stream launch (0 = one launch a batch)
    side_stream_min: int = 1 << 20        # pipelined batches of fewer channel samples stay on one stream (no events)


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


def _dist_world():
    """(rank, world) of the initialised process group, else (0, 1)."""
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return 0, 1
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(), dist.get_world_size()


def _dist_exchange(rank: int, world: int):
    """Exchange for one process per rank: every rank's per-batch error counts of one round, as a
    [world][k] list, through one all-reduce of a zero-padded float64 vector (integer counts < 2^53 add
    exactly). RCCL (``nccl``) reduces a device tensor, gloo a host one; an initialised group of size 1
    still runs the all-reduce (a 1-GPU ``nccl`` group exercises the device path)."""
    def exchange(local):
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return [list(local)]
        import torch
        k = len(local)
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.zeros(world * k, dtype=torch.float64, device=dev)
        t[rank * k:(rank + 1) * k] = torch.tensor([float(v) for v in local], dtype=torch.float64)
        dist.all_reduce(t)
        v = t.cpu().tolist()
        return [v[r * k:(r + 1) * k] for r in range(world)]
    return exchange


def global_batch(base: int, round_: int, rank: int, world: int) -> int:
    """Global index of the batch rank ``rank`` of ``world`` decodes in its local round ``round_`` of a point
    whose first global batch is ``base``: batches are dealt round-robin, g = base + round * world + rank, so
    the global order (rank 0's round 0, rank 1's round 0, ..., rank 0's round 1, ...) is the 1-rank order."""
    return int(base) + int(round_) * int(world) + int(rank)


class _SyncRunner:
    """The reference driver's call sequence, one batch at a time (DVB-S2/BER_simulation_OpenCL.py:105-112):
    ``quantize_direct_OpenCL[_LLR]`` -> ``decode_OpenCL*`` -> ``return_errors_all_zero`` (a host sync per batch).
    Used with ``cfg.pipeline=False`` and for decoder / quantiser objects that are not device-backed."""
    lookahead = False

    def __init__(self, decoder, kind, quanti, tx, B, N_var, pb_ch, pb_bits, err_rows, thr, cfg):
        self.decoder, self.kind, self.quanti, self.tx = decoder, kind, quanti, tx
        self.B, self.N_var, self.pb_ch, self.pb_bits = B, N_var, pb_ch, pb_bits
        self.err_rows, self.thr, self.cfg = err_rows, thr, cfg
        if tx is not None:
            import torch
            self.cnt = torch.zeros(1, dtype=torch.int64, device=tx.encoder.device)

    def enqueue(self, gs, next_g=None):
        from .engine import count_errors
        dec_, q, local = self.decoder, self.quanti, []
        for g in gs:
            kw = {}
            if self.tx is not None:
                self.tx.offset = g * self.pb_bits
                kw["bits"] = self.tx.transmit_bits()
            q.offset = g * self.pb_ch
            if self.kind == "ib":
                rec = q.quantize_direct_OpenCL(self.N_var, self.B, **kw)
                dec = dec_.decode_OpenCL(rec, buffer_in=True, return_buffer=True)
            else:
                rec = q.quantize_direct_OpenCL_LLR(self.N_var, self.B, dtype=self.cfg.llr_dtype, **kw)
                fn = dec_.decode_OpenCL_min_sum if self.kind == "minsum" else dec_.decode_OpenCL_belief_propagation
                dec = fn(rec, buffer_in=True, return_buffer=True)
            if self.tx is None:
                local.append(float(dec_.return_errors_all_zero(dec)))
            else:
                local.append(float(count_errors(dec.contiguous(), self.err_rows, self.thr, kw["bits"], self.cnt).item()))
        return local

    def read(self, handle):
        return handle

    def finish(self):
        pass


class _DeviceRunner:
    """Pipelined batches on one HIP device. Per batch k of a round: the side stream generates batch k+1's channel
    (``ibl_channel_sample`` with the quantiser's CDF / LLRs, seed and the batch's global Philox offset; encoded:
    ``ibl_random_bits`` + ``ibl_encode`` first) into the free half of a double buffer, once the decode that last
    read that half is done; the caller's stream waits for batch k's channel and decodes it through the drop-in
    method (``decode_OpenCL*``, return_buffer); the side stream then counts batch k's errors into slot k of a device
    vector (the rows and threshold ``return_errors_all_zero`` uses, or the transmitted bits). The host reads a
    round's vector once (``read``) — by then ``_rank_sweep`` has enqueued the next round. IB channels and decisions
    are u8 cluster ids (the reference's int32 holds the same values; a quarter of the bytes to write and count).
    Batches of fewer than ``cfg.side_stream_min`` channel samples (the reference DVB-S2 driver's msg_at_time = 2)
    have little to overlap and many short launches: they run on the caller's stream alone, in the same order and
    with the same per-round host read, without the cross-stream events."""
    lookahead = True

    def __init__(self, decoder, kind, quanti, tx, B, N_var, pb_ch, pb_bits, err_rows, thr, cfg):
        import torch
        self.torch = torch
        self.decoder, self.kind, self.quanti, self.tx = decoder, kind, quanti, tx
        self.B, self.pb_ch, self.pb_bits, self.err_rows, self.thr = B, pb_ch, pb_bits, err_rows, thr
        self.gen_chunk = int(cfg.gen_chunk)
        # u8 decisions from decoders whose decode_OpenCL takes out_dtype (this package's); others as they come
        self.dec_kw = {}
        if kind == "ib":
            import inspect
            try:
                if "out_dtype" in inspect.signature(decoder.decode_OpenCL).parameters:
                    self.dec_kw = {"out_dtype": torch.uint8}
            except (TypeError, ValueError):  # pragma: no cover - builtins without a signature
                pass
        dev = decoder.device
        self.dev = dev
        self.main = torch.cuda.current_stream(dev)
        self.single = N_var * B < int(cfg.side_stream_min)
        self.side = self.main if self.single else torch.cuda.Stream(dev)
        ch_dtype = torch.uint8 if kind == "ib" else (cfg.llr_dtype or torch.float64)
        with torch.cuda.stream(self.side):
            self.ch = [torch.empty((N_var, B), dtype=ch_dtype, device=dev) for _ in range(2)]
            if tx is not None:
                self.info = [torch.empty((tx.K, B), dtype=torch.uint8, device=dev) for _ in range(2)]
                self.code = [torch.empty((N_var, B), dtype=torch.uint8, device=dev) for _ in range(2)]
        if not self.single:
            self.side.wait_stream(self.main)    # the buffers exist before the side stream writes them
        self.used = [None, None]                # event: the decode that last read each half is done
        self.ready = [None, None]
        self.slot_g = [None, None]              # global batch whose channel a half holds (None: consumed)
        self.k = 0

    def _gen(self, slot, g):
        from .engine import channel_sample, random_bits
        torch, q = self.torch, self.quanti
        with torch.cuda.stream(self.side):
            if self.used[slot] is not None:     # (one stream: the decode precedes in stream order)
                self.side.wait_event(self.used[slot])
            bits = None
            if self.tx is not None:
                random_bits(self.info[slot], self.tx.seed, g * self.pb_bits)
                self.tx.encoder.encode_batch(self.info[slot], self.code[slot])
                bits = self.code[slot]
            # in row slices of ~gen_chunk samples: each slice is a short launch that can take the CUs in the gaps
            # between the decode's per-pass launches instead of holding the chip for the whole batch's sampling.
            # Slice rows start at multiples of 4, so every slice begins on a Philox block (4 samples): slice
            # [r0, r1) is the batch's stream from element r0 * B on, at counter g * pb_ch + r0 * B / 4.
            out = self.ch[slot]
            n, B = out.shape
            rows = n if self.gen_chunk <= 0 else max(4, (self.gen_chunk // max(B, 1)) // 4 * 4)
            llr = None if self.kind == "ib" else q.output_LLRs
            for r0 in range(0, n, rows):
                r1 = min(n, r0 + rows)
                channel_sample(out[r0:r1], q.cdf_t_given_x_equals_zero, q.seed, g * self.pb_ch + (r0 * B) // 4,
                               llr=llr, bits=None if bits is None else bits[r0:r1])
            ev = None
            if not self.single:
                ev = torch.cuda.Event()
                ev.record(self.side)
        self.ready[slot], self.slot_g[slot] = ev, g

    def enqueue(self, gs, next_g=None):
        from .engine import count_below, count_errors
        torch, d = self.torch, self.decoder
        with torch.cuda.stream(self.side):
            cnt = torch.zeros(len(gs), dtype=torch.int64, device=self.dev)
        for i, g in enumerate(gs):
            slot = self.k % 2
            if self.slot_g[slot] != g:
                self._gen(slot, g)
            ng = gs[i + 1] if i + 1 < len(gs) else next_g
            if ng is not None and self.slot_g[1 - slot] != ng:
                self._gen(1 - slot, ng)         # batch k+1's channel while batch k decodes
            if self.ready[slot] is not None:
                self.main.wait_event(self.ready[slot])
            with torch.cuda.stream(self.main):
                if self.kind == "ib":
                    dec = d.decode_OpenCL(self.ch[slot], buffer_in=True, return_buffer=True, **self.dec_kw)
                else:
                    fn = d.decode_OpenCL_min_sum if self.kind == "minsum" else d.decode_OpenCL_belief_propagation
                    dec = fn(self.ch[slot], buffer_in=True, return_buffer=True)
                ev = None
                if not self.single:
                    ev = torch.cuda.Event()
                    ev.record(self.main)
            self.used[slot], self.slot_g[slot] = ev, None
            with torch.cuda.stream(self.side):
                if ev is not None:
                    self.side.wait_event(ev)
                    dec.record_stream(self.side)
                if self.tx is None:
                    count_below(dec, self.err_rows, self.thr, out=cnt[i:i + 1])
                else:
                    count_errors(dec, self.err_rows, self.thr, self.code[slot], out=cnt[i:i + 1])
            self.k += 1
        done = torch.cuda.Event()
        done.record(self.side)
        return cnt, done

    def read(self, handle):
        cnt, done = handle
        done.synchronize()
        return [float(v) for v in cnt.cpu().tolist()]

    def finish(self):
        self.torch.cuda.synchronize(self.dev)


def _drain(ctx) -> None:
    """Synchronise `ctx` when it is a HIP device (pipelined batches of another emulated rank may be in flight)."""
    try:
        import torch
    except ImportError:  # pragma: no cover
        return
    if isinstance(ctx, torch.device) and ctx.type == "cuda":
        torch.cuda.synchronize(ctx)


def _device_backed(decoder, quanti) -> bool:
    dev = getattr(decoder, "device", None)
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(dev, torch.device) and dev.type == "cuda" and hasattr(quanti, "cdf_t_given_x_equals_zero")


def _rank_sweep(decoder, cfg: BERConfig, quantizer_factory, rank: int, world: int, log):
    """The Eb/N0 sweep of one rank as a generator: it yields the error counts of the batches it decoded in
    one exchange (``sync_every`` rounds) and is sent back the [world][sync_every] counts of every rank.

    Channel (and, in encoded mode, bit) streams are keyed on the GLOBAL batch index g (``global_batch``):
    batch g's Philox counter starts at g * philox_blocks(N, B) under key ``cfg.seed`` — the reference draws
    one stream per batch (AWGN_Quantizer_BPSK.py:201-248) and so does the 1-rank run, batch after batch.
    Each rank then walks the exchanged counts in global order and applies the reference's loop condition
    (``while errors < min_errors``, ``DVB-S2/BER_simulation_OpenCL.py:115-121``, plus ``max_blocks``)
    before each batch; the batches after the stop are discarded (at most world * sync_every - 1 per point, and
    the device runner's one round of lookahead) and the next point starts at the first unused global index. A
    k-rank sweep therefore counts exactly the frames, errors and blocks of the 1-rank sweep with the same
    per-rank batch, whatever k and ``sync_every`` are."""
    from .awgn_quantizer import AWGN_Channel_Quantizer
    from .engine import philox_blocks
    kind = decoder_kind(decoder)
    N_var = int(decoder.codeword_len)
    R_c = float(decoder.R_c)
    B = int(cfg.msg_at_time)
    S = max(1, int(cfg.sync_every))
    if quantizer_factory is None:
        def quantizer_factory(s2):
            return AWGN_Channel_Quantizer(s2, cfg.AD_max_abs, cfg.cardinality_T_channel, cfg.cardinality_Y_channel)
    ebn0 = [float(cfg.EbN0_dB_start)]
    ber: List[float] = [0.0]
    res = BERResult(np.array([]), np.array([]))
    pb_ch = philox_blocks(N_var, B)
    base = 0                                    # first global batch of the current point
    tx, pb_bits = None, 0
    # rows return_errors_all_zero counts: all N for the regular IB class (:297-300), data_len otherwise
    err_rows = N_var if type(decoder).__name__ == "Discrete_LDPC_Decoder_class" else int(getattr(decoder, "data_len", N_var))
    thr = getattr(decoder, "cardinality_T_decoder_ops", 16) // 2 if kind == "ib" else 0.0
    if cfg.encoded:
        from .ldpc_encoder import LDPC_BPSK_Transmitter
        tx = LDPC_BPSK_Transmitter(decoder.H_sparse, B, seed=int(cfg.seed), device=getattr(decoder, "device", None))
        pb_bits = philox_blocks(tx.K, B)

    def more(errors, blocks):
        return errors < cfg.min_errors and (cfg.max_blocks is None or blocks < cfg.max_blocks)

    while True:
        EbN0_dB = ebn0[-1]
        sigma_n2 = 10 ** (-EbN0_dB / 10) / (2 * R_c)
        quanti = quantizer_factory(sigma_n2)
        quanti.seed = int(cfg.seed)
        quanti.offset = base * pb_ch
        quanti.init_OpenCL_quanti(N_var, B, return_buffer_only=True, context_=getattr(decoder, "device", None))
        _drain(quanti.context)     # a decoder shared by emulated ranks is rebuilt here: nothing may still use it
        decoder.init_OpenCL_decoding(B, quanti.context)
        run_cls = _DeviceRunner if (cfg.pipeline and _device_backed(decoder, quanti)) else _SyncRunner
        runner = run_cls(decoder, kind, quanti, tx, B, N_var, pb_ch, pb_bits, err_rows, thr, cfg)
        errors, blocks, used, rnd = 0.0, 0, 0, 0
        t0 = time.time()

        def round_of(r):
            """This rank's global batches of local rounds r .. r+S-1, and the first batch of the round after (its
            channel is generated while the round's last batch decodes) unless max_blocks ends the point first."""
            nxt = None if (cfg.max_blocks is not None and (r + S) * world * B >= cfg.max_blocks) \
                else global_batch(base, r + S, rank, world)
            return [global_batch(base, r + s, rank, world) for s in range(S)], nxt

        pending = runner.enqueue(*round_of(rnd)) if more(errors, blocks) else None
        while more(errors, blocks):
            nxt = None
            # the next round goes to the device before this round's counts are read, unless max_blocks already
            # ends the point with this round
            if runner.lookahead and (cfg.max_blocks is None or blocks + S * world * B < cfg.max_blocks):
                nxt = runner.enqueue(*round_of(rnd + S))
            local = runner.read(pending)
            counts = yield local
            stop = False
            for s in range(S):                  # global order: round-major, rank-minor
                for r in range(world):
                    if not more(errors, blocks):
                        stop = True
                        break
                    errors += counts[r][s]      # integer counts, summed exactly in float64
                    blocks += B
                    used += 1
                if stop:
                    break
            rnd += S
            pending = nxt if nxt is not None else (runner.enqueue(*round_of(rnd)) if more(errors, blocks) else None)
        runner.finish()
        base += used
        spent = time.time() - t0
        ber[-1] = errors / (R_c * blocks * N_var) if blocks else 0.0
        res.errors.append(errors)
        res.blocks.append(blocks)
        res.seconds.append(spent)
        if log and rank == 0:
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


def _drive(gens, exchange):
    """Run rank generators in lockstep: each round's local counts go through ``exchange`` (a list of the
    gens' lists -> the [world][k] matrix) and the matrix is sent back to every gen."""
    locals_, done = [], []
    for g in gens:      # a sweep that decodes nothing (min_errors <= 0, max_blocks <= 0) returns before a yield
        try:
            locals_.append(next(g))
        except StopIteration as e:
            done.append(e.value)
    if done:
        if len(done) != len(gens):
            raise RuntimeError("ranks of a BER sweep disagree on when to stop")
        return done
    while True:
        counts = exchange(locals_)
        nxt, done = [], []
        for g in gens:
            try:
                nxt.append(g.send(counts))
            except StopIteration as e:
                done.append(e.value)
        if done:
            if len(done) != len(gens):
                raise RuntimeError("ranks of a BER sweep disagree on when to stop")
            return done
        locals_ = nxt


def run_ber(decoder, cfg: BERConfig, quantizer_factory: Optional[Callable] = None,
            log: Optional[Callable[[str], None]] = None, rank: Optional[int] = None,
            world: Optional[int] = None) -> BERResult:
    """Run the Eb/N0 sweep with ``decoder`` (a drop-in decoder instance). ``quantizer_factory(sigma_n2)``
    returns a quantiser object with the reference methods (default: :class:`.awgn_quantizer.AWGN_Channel_Quantizer`
    with ``cfg.cardinality_T_channel`` clusters). ``rank`` / ``world`` default to the initialised process
    group (one process per GPU; counters exchanged by all-reduce) or (0, 1). The result is the same for
    every world size (see ``_rank_sweep``); :func:`run_ber_lockstep` emulates k ranks in one process."""
    r0, w0 = _dist_world()
    rank = r0 if rank is None else int(rank)
    world = w0 if world is None else int(world)
    if world > 1 and w0 != world:
        raise ValueError(f"world={world} needs an initialised process group of that size (have {w0}); "
                         "use run_ber_lockstep to emulate ranks in one process")
    gen = _rank_sweep(decoder, cfg, quantizer_factory, rank, world, log)
    ex = _dist_exchange(rank, world)
    return _drive([gen], lambda loc: ex(loc[0]))[0]


def run_ber_lockstep(decoders, cfg: BERConfig, world: int, quantizer_factory: Optional[Callable] = None,
                     log: Optional[Callable[[str], None]] = None) -> BERResult:
    """``world`` ranks of a multi-GPU sweep emulated in one process: rank r decodes its global batches with
    ``decoders[r]`` (or one shared decoder; a decode call is self-contained), rounds run in lockstep and
    the counts are exchanged in memory. Returns rank 0's result (every rank's is checked equal)."""
    decs = list(decoders) if isinstance(decoders, (list, tuple)) else [decoders] * int(world)
    if len(decs) != world:
        raise ValueError("one decoder per rank")
    gens = [_rank_sweep(decs[r], cfg, quantizer_factory, r, world, log) for r in range(world)]
    out = _drive(gens, lambda loc: [list(x) for x in loc])
    for o in out[1:]:
        if o.errors != out[0].errors or o.blocks != out[0].blocks:
            raise RuntimeError("emulated ranks disagree")
    return out[0]
