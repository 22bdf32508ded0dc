"""BER-curve parity (north_star: "BER curves matching the reference path at every Eb/N0 point").

The BER driver (``ber.run_ber``: the Eb/N0 state machine of ``DVB-S2/BER_simulation_OpenCL.py:101-143``,
device channel generation, the drop-in decoder with its batch-global early stop,
``return_errors_all_zero``) is replayed on the CPU: the same state machine over the identical Philox
channel stream (``oracle.channel_sample``), decoded by the oracle (``oracle.ib_decode`` /
``oracle.float32_decode``, early stop on, as ``decode_OpenCL*`` do). Bar: identical Eb/N0 points,
per-point error and block counts, and BER vectors.

Table values: discrete-density-evolution tables (``tables.de_tables``, per-iteration alphabets and
matching, round 6) stand in for the reference's IB-designed ``.pkl`` tables, which need the absent
``ib_base`` package — parity with the published decoders' curves is unpinned; parity here is HIP path
vs oracle on the same tables and channel.
"""
import numpy as np
import pytest
import torch

from informationbottleneckdecodingldpc_amd import codes, engine, graph, tables
from informationbottleneckdecodingldpc_amd.awgn_quantizer import AWGN_Channel_Quantizer
from informationbottleneckdecodingldpc_amd.ber import BERConfig, run_ber
from oracle import oracle

pytestmark = pytest.mark.gpu


def _quanti(cfg, s2):
    return AWGN_Channel_Quantizer(s2, cfg.AD_max_abs, cfg.cardinality_T_channel, cfg.cardinality_Y_channel)


def _replay(cfg, n_v, data_len, R_c, decode, errors_of):
    """run_ber's state machine (ber.py, reference :101-173) with the oracle as the decoder."""
    ebn0, ber, errs, blks = [float(cfg.EbN0_dB_start)], [0.0], [], []
    offset = 0
    while True:
        s2 = 10 ** (-ebn0[-1] / 10) / (2 * R_c)
        q = _quanti(cfg, s2)
        errors, blocks = 0.0, 0
        while errors < cfg.min_errors and (cfg.max_blocks is None or blocks < cfg.max_blocks):
            cl = oracle.channel_sample(q.cdf_t_given_x_equals_zero, cfg.seed, offset, n_v, cfg.msg_at_time)
            offset += engine.philox_blocks(n_v, cfg.msg_at_time)
            errors += errors_of(decode(cl, q), data_len)
            blocks += cfg.msg_at_time
        ber[-1] = errors / (R_c * blocks * n_v)
        errs.append(errors)
        blks.append(blocks)
        if ber[-1] > cfg.target_error_rate and ebn0[-1] < cfg.EbN0_dB_max_value:
            step = cfg.EbN0_dB_small_stepwidth if ber[-1] < cfg.BER_go_on_in_smaller_steps \
                else cfg.EbN0_dB_normal_stepwidth
            ebn0.append(ebn0[-1] + step)
            ber.append(0.0)
        else:
            break
    return np.asarray(ebn0), np.asarray(ber), errs, blks


def _assert_same(r, ref):
    ebn0, ber, errs, blks = ref
    np.testing.assert_allclose(r.EbN0_dB_vector, ebn0, rtol=0, atol=1e-12)
    assert [int(e) for e in r.errors] == [int(e) for e in errs]
    assert r.blocks == blks
    np.testing.assert_array_equal(r.BER_vector, ber)
    assert len(ebn0) >= 3


@pytest.mark.parametrize("name,imax,B,max_blocks,start,stop,step", [
    ("wlan", 20, 256, 1024, 0.5, 2.0, 0.5),           # WLAN N=1296 (the reference's own generator)
    ("dvbs2", 20, 32, 64, 1.0, 2.0, 0.5),             # DVB-S2 N=64800, small batches
])
def test_ib_ber_curve_equals_oracle(name, imax, B, max_blocks, start, stop, step, wlan_H, dvb_H):
    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import \
        Discrete_LDPC_Decoder_class_irregular
    H = wlan_H if name == "wlan" else dvb_H
    g = graph.build_graph(H)
    cfg = BERConfig(EbN0_dB_start=start, EbN0_dB_max_value=stop, EbN0_dB_normal_stepwidth=step,
                    EbN0_dB_small_stepwidth=step / 2, target_error_rate=1e-9, min_errors=10 ** 9,
                    msg_at_time=B, max_blocks=max_blocks, seed=11)
    design = _quanti(cfg, 10 ** (-1.5 / 10) / (2 * g.R_c))       # tables designed at 1.5 dB
    rho, lam = tables.edge_degree_distributions(g)               # per-iteration DE alphabets (round 6)
    tb = tables.de_tables(design.p_t_given_x_equals_zero, design.output_LLRs, rho, lam, imax)
    dec = Discrete_LDPC_Decoder_class_irregular(H, imax, 16, 16, tb.cn, tb.vn, tb.match_cn, tb.match_vn, B,
                                                match="true")
    r = run_ber(dec, cfg)
    ref = _replay(cfg, g.n_v, dec.data_len, float(dec.R_c),
                  lambda cl, q: oracle.ib_decode(g, tb, cl, match=True, early_stop=True),
                  lambda out, dl: float((out[:dl] < 8).sum()))
    _assert_same(r, ref)
    assert ref[2][0] > ref[2][-1]          # the curve falls over the sweep


@pytest.mark.parametrize("prec", [torch.float64, torch.float32])
def test_bp_ber_curve_c5_dvbs2(prec, dvb_H):
    """BASELINE C5 (DVB-S2 BP, i_max=100, Eb/N0 sweep) through the reference-named BP class and the BER
    driver, as ``WLAN/BER_simulation_OpenCL_quant_BP.py:105-110`` calls it (``quantize_direct_OpenCL_LLR`` ->
    ``decode_OpenCL_belief_propagation`` -> ``return_errors_all_zero``), replayed on the fp64 oracle
    (``oracle.float_decode(kind=BP)``, early stop on) over the identical Philox channel stream.

    Bar: identical Eb/N0 points and block counts (the state machine), and per-point error counts
    identical to the oracle's — for the fp64 build always; for the fp32 build where the two
    trajectories agree (every converged codeword does: H5, test_gpu_float.py), otherwise within the
    stated bound |e32 - e64| <= 4 sqrt(e32 + e64 + 1) per point (a paired-difference bound, ~6e-5
    false-alarm rate under 'same decoder statistic'). Measured on MI355X: identical counts at every
    point for both builds (DESIGN.md §Float parity)."""
    from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular
    g = graph.build_graph(dvb_H)
    B, imax = 16, 100
    bp = BeliefPropagationDecoderClassIrregular(dvb_H, imax, 16, B, precision=prec)
    cfg = BERConfig(EbN0_dB_start=0.2, EbN0_dB_max_value=1.2, EbN0_dB_normal_stepwidth=0.25,
                    EbN0_dB_small_stepwidth=0.125, target_error_rate=1e-9, min_errors=10 ** 9, msg_at_time=B,
                    max_blocks=32, seed=23, llr_dtype=prec)
    r = run_ber(bp, cfg)
    np_dt = np.float64 if prec == torch.float64 else np.float32

    def decode(cl, q):
        llr = q.output_LLRs.astype(np_dt)[cl].astype(np.float64)   # the build's input LLRs, exactly
        return oracle.float_decode(g, oracle.BP, imax, llr, early_stop=True)
    ref = _replay(cfg, g.n_v, bp.data_len, float(bp.R_c), decode, lambda out, dl: float((out[:dl] < 0).sum()))
    ebn0, ber, errs, blks = ref
    np.testing.assert_allclose(r.EbN0_dB_vector, ebn0, rtol=0, atol=1e-12)
    assert len(ebn0) >= 3 and r.blocks == blks
    got = [int(e) for e in r.errors]
    want = [int(e) for e in errs]
    print(f"BP {prec}: points {list(ebn0)} errors gpu {got} oracle {want}")
    if prec == torch.float64:
        assert got == want
        np.testing.assert_array_equal(r.BER_vector, ber)
    else:
        for a_, b_ in zip(got, want):
            assert abs(a_ - b_) <= 4 * np.sqrt(a_ + b_ + 1), (got, want)
    assert want[0] > want[-1]              # the curve falls over the sweep


def test_minsum_fp32_ber_curve_equals_oracle():
    """BASELINE C3's code and decoder (WLAN N=1944, min-sum fp32, fused on-chip path) with the
    channel's float32 cluster LLRs: the BER curve equals the fp32 oracle's."""
    from informationbottleneckdecodingldpc_amd.min_sum_decoder_irreg import Min_Sum_Decoder_class_irregular
    H = codes.wlan_80211n(81)
    g = graph.build_graph(H)
    B = 512
    dec = Min_Sum_Decoder_class_irregular(H, 30, 16, B)
    cfg = BERConfig(EbN0_dB_start=1.0, EbN0_dB_max_value=3.0, EbN0_dB_normal_stepwidth=1.0,
                    EbN0_dB_small_stepwidth=0.5, target_error_rate=1e-9, min_errors=10 ** 9, msg_at_time=B,
                    max_blocks=1024, seed=5, llr_dtype=torch.float32)
    r = run_ber(dec, cfg)

    def decode(cl, q):
        llr = q.output_LLRs.astype(np.float32)[cl]
        return oracle.float32_decode(g, 30, llr, early_stop=True)
    ref = _replay(cfg, g.n_v, dec.data_len, float(dec.R_c), decode, lambda out, dl: float((out[:dl] < 0).sum()))
    _assert_same(r, ref)


def test_bp_c5_sweep_world_size_invariant(dvb_H):
    """C5's BP sweep (DVB-S2, i_max=100, fp64, B=8) as an emulated 2-rank run (``run_ber_lockstep``: rank 0
    and rank 1 decode global batches 2j and 2j+1, counters exchanged per round) and as a 3-rank run with
    two rounds per exchange equals the 1-rank sweep and the oracle replay point for point. min_errors
    stops the first points inside a round (the extra batches are discarded), max_blocks = 5 batches the
    later ones — neither is a multiple of the world size (``ber._rank_sweep``)."""
    from informationbottleneckdecodingldpc_amd.ber import run_ber_lockstep
    from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular
    g = graph.build_graph(dvb_H)
    B, imax = 8, 100
    bp = BeliefPropagationDecoderClassIrregular(dvb_H, imax, 16, B, precision=torch.float64)
    cfg = BERConfig(EbN0_dB_start=0.2, EbN0_dB_max_value=1.2, EbN0_dB_normal_stepwidth=0.4,
                    EbN0_dB_small_stepwidth=0.2, target_error_rate=1e-9, min_errors=20000, msg_at_time=B,
                    max_blocks=40, seed=31, llr_dtype=torch.float64)
    one = run_ber(bp, cfg)
    two = run_ber_lockstep(bp, cfg, 2)
    cfg3 = BERConfig(**{**cfg.__dict__, "sync_every": 2})
    three = run_ber_lockstep(bp, cfg3, 3)

    def decode(cl, q):
        return oracle.float_decode(g, oracle.BP, imax, q.output_LLRs[cl], early_stop=True)
    ref = _replay(cfg, g.n_v, bp.data_len, float(bp.R_c), decode, lambda out, dl: float((out[:dl] < 0).sum()))
    print(f"C5 world-invariance: points {list(ref[0])} errors {ref[2]} blocks {ref[3]}")
    for r in (one, two, three):
        _assert_same(r, ref)
    assert ref[3][0] < cfg.max_blocks and ref[3][-1] == cfg.max_blocks   # both stop rules exercised


@pytest.mark.parametrize("side", [0, None])   # 0: side stream at every batch size; None: the default threshold
@pytest.mark.parametrize("case", ["ib", "ib_encoded", "bp32", "lockstep2"])
def test_pipelined_driver_equals_sync_driver(case, side, wlan_H, dvb_H):
    """the pipelined BER driver (``_DeviceRunner``: channel of batch k+1 generated on a side stream
    into a double buffer while batch k decodes, error counts on the side stream, counts read once per round with the
    next round already enqueued) counts exactly the frames and errors of the reference call sequence
    (``cfg.pipeline=False``: quantise -> decode -> return_errors_all_zero per batch) — min_errors stops inside a
    round (the lookahead round is discarded), max_blocks ends the last points; encoded codewords; BP fp32; two
    emulated ranks sharing one decoder. Both pipelined modes: side stream + events, and (batches below
    ``side_stream_min``, as these are by default) the caller's stream alone."""
    from informationbottleneckdecodingldpc_amd.ber import run_ber_lockstep
    from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular
    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import \
        Discrete_LDPC_Decoder_class_irregular
    H = dvb_H if case == "bp32" else wlan_H
    g = graph.build_graph(H)
    B = 8 if case == "bp32" else 64
    kw = dict(EbN0_dB_start=0.5, EbN0_dB_max_value=2.0, EbN0_dB_normal_stepwidth=0.5, EbN0_dB_small_stepwidth=0.25,
              target_error_rate=1e-9, min_errors=3000 if case != "bp32" else 20000, msg_at_time=B,
              max_blocks=20 * B, seed=17, sync_every=3, encoded=case == "ib_encoded")
    if case == "bp32":
        dec = BeliefPropagationDecoderClassIrregular(H, 30, 16, B, precision=torch.float32)
        kw["llr_dtype"] = torch.float32
        kw["EbN0_dB_max_value"], kw["EbN0_dB_normal_stepwidth"] = 1.0, 0.25
    else:
        design = _quanti(BERConfig(), 10 ** (-1.5 / 10) / (2 * g.R_c))
        tb = tables.llr_tables(design.output_LLRs, g.d_c_max, g.d_v_max, 15)
        dec = Discrete_LDPC_Decoder_class_irregular(H, 15, 16, 16, tb.cn, tb.vn, tb.match_cn, tb.match_vn, B,
                                                    match="true")
    res = {}
    if side is not None:
        kw["side_stream_min"] = side
    for pipe in (True, False):
        cfg = BERConfig(**kw, pipeline=pipe)
        res[pipe] = run_ber_lockstep(dec, cfg, 2) if case == "lockstep2" else run_ber(dec, cfg)
    a, b = res[True], res[False]
    print(f"{case}: points {list(b.EbN0_dB_vector)} errors {b.errors} blocks {b.blocks}")
    assert a.errors == b.errors and a.blocks == b.blocks
    np.testing.assert_array_equal(a.BER_vector, b.BER_vector)
    np.testing.assert_array_equal(a.EbN0_dB_vector, b.EbN0_dB_vector)
    assert len(b.blocks) >= 3 and b.blocks[0] < kw["max_blocks"] and b.blocks[-1] == kw["max_blocks"]
