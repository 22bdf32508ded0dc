"""GPU parity of the information-bottleneck decoder (HIP kernels via the C ABI) against the CPU
oracle (oracle/ib_oracle.c, itself pinned to the reference's decode_on_host by
tests/test_cpu_oracle.py) and against the reference's own golden outputs.

Bar: bit-exact cluster ids and identical stop iteration.
"""
import numpy as np
import pytest
import torch

from informationbottleneckdecodingldpc_amd import codes, graph, tables
from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0
from oracle import oracle
from tests._codes import mixed_code as _mixed_code

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def eng():
    from informationbottleneckdecodingldpc_amd import engine
    return engine


def _run(eng, g_edges, tb, ch, match, early, out_dtype=torch.int32, ch_dtype=torch.int32, force_generic=False,
         graph_obj=None, path="auto", small_b=None, max_batch=None):
    G = graph_obj or eng.Graph(g_edges, DEV)
    dec = eng.IBDecoder(G, tb, match, max_batch=max_batch or ch.shape[1], force_generic=force_generic, path=path)
    if small_b is not None:
        dec.small_batch = small_b
    it = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = dec.decode(torch.from_numpy(ch).to(DEV).to(ch_dtype).contiguous(), out_dtype=out_dtype,
                     early_stop=early, iters=it)
    torch.cuda.synchronize()
    return out.cpu().numpy().astype(np.int32), int(it.item()), dec


def test_decode_ignores_diagnostic_environment(eng, dvb_H, monkeypatch):
    """IBL_VN_PART made every per-pass decode skip part of the variable pass. The product
    library has no such hook any more (diagnostic builds only), so a decode with it set — and with the other
    timing-only variables set — still equals the oracle."""
    monkeypatch.setenv("IBL_VN_PART", "heavy")
    monkeypatch.setenv("IBL_TRACE_WAVES", "/nonexistent/trace")
    monkeypatch.setenv("IBL_TRACE_FUSED", "/nonexistent/ftrace")
    g = graph.build_graph(dvb_H)
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, 4, seed=3)
    ch = np.random.default_rng(3).integers(0, 16, (g.n_v, 9)).astype(np.int32)
    ref = oracle.ib_decode(g, tb, ch, match=True, early_stop=False)
    out, _, dec = _run(eng, g, tb, ch, True, False, path="passes")
    assert dec.fast_path
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("name,imax,B,match,early,ebn0", [
    ("dvb", 6, 2, True, False, None),        # the reference DVB-S2 driver's msg_at_time
    ("dvb", 20, 2, True, True, 3.0),         # converging: early stop before imax-1
    ("dvb", 5, 33, False, True, None),       # ragged last word
    ("dvb", 4, 130, True, False, None),      # 17 words, forced onto the small kernels
    ("mixed16", 6, 9, False, True, None),    # every body of the MAXD=16 instantiations (degrees 2..16 / 1..16)
    ("mixed8", 7, 64, True, True, 4.0)])     # MAXD=8 bodies with matching, converging
def test_ib_small_batch_kernels(eng, name, imax, B, match, early, ebn0, dvb_H):
    """The small-batch per-pass kernels (ib_*_small: wave item = up to 64 same-degree nodes x 8 codewords) and
    the fast kernels (wave item = one node x 1024 codewords) both equal the oracle at small B, with the same
    stop iteration; u8 and i32 in and out; a decoder sized for a larger max_batch (wider rows) too."""
    H = {"dvb": lambda: dvb_H,
         "mixed16": lambda: _mixed_code(np.arange(2, 17), np.arange(1, 17), 600, seed=15),
         "mixed8": lambda: _mixed_code(np.array([3, 5, 6, 7, 8]), np.array([2, 3, 5, 6, 7, 8]), 500, seed=5)}[name]()
    g = graph.build_graph(H)
    G = eng.Graph(g, DEV)
    if ebn0 is None:
        tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, imax, seed=B + imax)
        ch = np.random.default_rng(B).integers(0, 16, (g.n_v, B)).astype(np.int32)
    else:
        q = UniformQuantizer(sigma2_from_ebn0(ebn0, g.R_c), 16)
        tb = tables.llr_tables(q.output_LLRs, g.d_c_max, g.d_v_max, imax)
        ch = q.sample_all_zero(g.n_v, B, np.random.default_rng(B)).astype(np.int32)
    ref, ref_it = oracle.ib_decode(g, tb, ch, match=match, early_stop=early, return_iters=True)
    if name == "dvb" and ebn0 is not None and early:
        assert ref_it < imax - 1            # the batch-global stop happens inside the loop
    for small_b, mb, dt in ((1024, None, torch.int32), (1024, 5000, torch.uint8), (0, None, torch.int32)):
        out, it, dec = _run(eng, g, tb, ch, match, early, path="passes", small_b=small_b, max_batch=mb,
                            out_dtype=dt, ch_dtype=dt)
        assert dec.fast_path and not dec.fused and dec.small_batch == small_b
        assert it == ref_it, (small_b, mb)
        np.testing.assert_array_equal(out, ref, err_msg=f"small_b={small_b} max_batch={mb}")


def test_ib_small_batch_default_and_generic(eng, wlan_H):
    """Default threshold 224 (measured crossover); the generic path refuses the small-batch kernels."""
    g = graph.build_graph(wlan_H)
    G = eng.Graph(g, DEV)
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, 3)
    assert eng.IBDecoder(G, tb, True, 16, path="passes").small_batch == 224
    gen = eng.IBDecoder(G, tb, True, 16, force_generic=True)
    assert gen.small_batch == 0
    from informationbottleneckdecodingldpc_amd._lib import IBLError
    with pytest.raises(IBLError):
        gen.small_batch = 8


CASES = [
    # name, imax, B, match, early
    ("wlan", 1, 3, False, False),
    ("wlan", 2, 5, True, False),
    ("wlan", 10, 300, True, False),
    ("wlan", 10, 257, False, True),
    ("reg", 6, 64, False, False),
    ("reg", 5, 511, True, True),
    ("dvb", 4, 6, True, False),
    ("dvb", 3, 2, False, True),
    # B past one 2048-codeword light-row chunk (the variable pass's degree <= 4 items read 1-KiB row
    # segments; rows are padded to 2048 codewords): a full chunk plus a ragged one
    ("reg", 4, 3000, True, False),
    ("dvb", 2, 2100, False, True),
]


def _code(name, wlan_H, reg_H, dvb_H):
    return {"wlan": wlan_H, "reg": reg_H, "dvb": dvb_H}[name]


@pytest.mark.parametrize("name,imax,B,match,early", CASES)
@pytest.mark.parametrize("mode", ["auto", "passes", "generic"])
def test_ib_random_tables_vs_oracle(eng, name, imax, B, match, early, mode, wlan_H, reg_H, dvb_H):
    """Every path against the oracle: auto (fused on-chip kernel for WLAN / regular, per-pass for
    DVB-S2), per-pass fast kernels, generic reference-indexing kernels."""
    g = graph.build_graph(_code(name, wlan_H, reg_H, dvb_H))
    T = 16
    tb = tables.random_tables(T, T, g.d_c_max, g.d_v_max, imax, seed=imax * 7 + B)
    rng = np.random.default_rng(B)
    ch = rng.integers(0, T, (g.n_v, B)).astype(np.int32)
    ref, ref_it = oracle.ib_decode(g, tb, ch, match=match, early_stop=early, return_iters=True)
    generic = mode == "generic"
    out, it, dec = _run(eng, g, tb, ch, match, early, force_generic=generic, path="passes" if generic else mode)
    assert dec.fast_path == (not generic)
    assert dec.fused == (mode == "auto" and name != "dvb")
    assert it == ref_it
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("ch_dtype,out_dtype", [(torch.uint8, torch.uint8), (torch.uint8, torch.int32),
                                                (torch.int32, torch.uint8)])
@pytest.mark.parametrize("B", [1, 4, 7, 256, 1030])
def test_ib_dtypes_and_ragged_batches(eng, wlan_H, ch_dtype, out_dtype, B):
    g = graph.build_graph(wlan_H)
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, 4, seed=5)
    ch = np.random.default_rng(B).integers(0, 16, (g.n_v, B)).astype(np.int32)
    ref = oracle.ib_decode(g, tb, ch, match=True)
    out, _, _ = _run(eng, g, tb, ch, True, False, out_dtype=out_dtype, ch_dtype=ch_dtype)
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("Tc,T", [(16, 8), (8, 8), (4, 16), (32, 32)])
def test_ib_other_alphabets(eng, reg_H, Tc, T):
    """T_ch != T_dec and T_dec > 16 run the generic path; T == T_ch <= 16 the fast path."""
    g = graph.build_graph(reg_H)
    imax = 4
    tb = tables.random_tables(Tc, T, g.d_c_max, g.d_v_max, imax, seed=Tc + T)
    ch = np.random.default_rng(1).integers(0, Tc, (g.n_v, 37)).astype(np.int32)
    ref = oracle.ib_decode(g, tb, ch, match=True)
    out, _, dec = _run(eng, g, tb, ch, True, False)
    assert dec.fast_path == (Tc == T and T <= 16)
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("match,cdegs,vdegs,fast", [
    (False, list(range(2, 17)), list(range(1, 17)), True),       # every body, MAXD=16 path on both sides
    (True, [3, 5, 6, 7, 8], [1, 2, 3, 5, 6, 7, 8], True),         # MAXD=8, every column-fetch degree, matching
    # matching, 9 variable degrees up to 12: 10 fold + 9 composed tables = 5 LDS regions (160 KiB) plus
    # the work counters exceed the CU's LDS, so the decoder takes the generic path (still bit-exact)
    (True, [2, 4, 6, 10], [2, 4, 6, 7, 12], False),
])
@pytest.mark.parametrize("early", [False, True])
def test_ib_mixed_degrees_fast_path(eng, match, cdegs, vdegs, fast, early):
    g = graph.build_graph(_mixed_code(np.array(cdegs), np.array(vdegs), 600, seed=len(cdegs)))
    imax, B = 7, 1100
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, imax, seed=len(vdegs))
    ch = np.random.default_rng(9).integers(0, 16, (g.n_v, B)).astype(np.int32)
    ref, ref_it = oracle.ib_decode(g, tb, ch, match=match, early_stop=early, return_iters=True)
    out, it, dec = _run(eng, g, tb, ch, match, early)
    assert dec.fast_path == fast
    assert it == ref_it
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("name,imax,B,match,early,ebn0", [
    ("reg8000", 50, 300, False, False, None),     # BASELINE C1/C2 code, ragged batch
    ("reg8000", 12, 64, False, True, 3.0),        # converging: stop before imax-1 (pass 2 re-run)
    ("wlan1944", 20, 1001, True, True, None),     # random tables never converge: one pass
    ("wlan", 9, 17, True, False, None),
    ("mixed16", 6, 130, False, True, None),       # every node body (degrees 2..16 / 1..16), MAXD=16
    ("mixed8", 7, 250, True, True, 4.0)])         # MAXD=8 bodies with matching, converging
def test_ib_fused_equals_passes_and_oracle(eng, name, imax, B, match, early, ebn0, wlan_H, monkeypatch):
    """The fused on-chip IB kernel (8 codewords per workgroup in LDS for all iterations, or 4 — the
    half groups small batches run, forced both ways with IBL_FUSED_NCW) equals the per-pass path and the
    oracle bit for bit, with the same stop iteration."""
    H = {"reg8000": lambda: codes.regular_code(8000, 3, 6, seed=0), "wlan1944": lambda: codes.wlan_80211n(81),
         "wlan": lambda: wlan_H,
         "mixed16": lambda: _mixed_code(np.arange(2, 17), np.arange(1, 17), 600, seed=15),
         "mixed8": lambda: _mixed_code(np.array([3, 5, 6, 7, 8]), np.array([2, 3, 5, 6, 7, 8]), 500, seed=5)}[name]()
    g = graph.build_graph(H)
    G = eng.Graph(g, DEV)
    if ebn0 is None:
        tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, imax, seed=B)
        ch = np.random.default_rng(B).integers(0, 16, (g.n_v, B)).astype(np.int32)
    else:
        q = UniformQuantizer(sigma2_from_ebn0(ebn0, g.R_c), 16)
        tb = tables.llr_tables(q.output_LLRs, g.d_c_max, g.d_v_max, imax)
        ch = q.sample_all_zero(g.n_v, B, np.random.default_rng(B)).astype(np.int32)
    ref, ref_it = oracle.ib_decode(g, tb, ch, match=match, early_stop=early, return_iters=True)
    for ncw in ("8", "4"):
        monkeypatch.setenv("IBL_FUSED_NCW", ncw)
        fo, fit, fdec = _run(eng, g, tb, ch, match, early, graph_obj=G, path="fused", out_dtype=torch.uint8,
                             ch_dtype=torch.uint8)
        assert fdec.fused
        # the group size that actually ran (a forced NCW=4 must not silently fall back to 8);
        # the MAXD=16 bodies may lack a half-group kernel under the whole-group launch bounds
        if ncw == "8" or name != "mixed16":
            assert fdec.fused_ncw(B) == int(ncw), (name, ncw)
        assert fit == ref_it, ncw
        np.testing.assert_array_equal(fo, ref, err_msg=f"IBL_FUSED_NCW={ncw}")
    po, pit, pdec = _run(eng, g, tb, ch, match, early, graph_obj=G, path="passes")
    assert not pdec.fused
    assert pit == ref_it
    if name == "reg8000" and early:
        assert ref_it < imax - 1
    np.testing.assert_array_equal(po, ref)


@pytest.mark.parametrize("name", ["reg8000", "wlan", "reg39"])
def test_ib_fused_table_sets(eng, name, wlan_H, monkeypatch):
    """Both table-staging modes of the fused kernel (two LDS table sets where they fit, as for the
    (3,6) N=8000 code — one quad of tables a pass, the sets in the two halves of one 64-KiB super-region —
    and the (3,9) N=900 code — two quads a pass, the second set one super-region up; one set + raw buffer
    otherwise, forced with IBL_FUSED_DBUF=0) equal the oracle;
    B = 4100 gives 513 groups of 8 codewords (a ragged last one), so workgroups run 2-3 groups and the
    set parity carries across the group boundary (also with 4-codeword half groups: 1025 workgroup
    groups)."""
    H = {"reg8000": lambda: codes.regular_code(8000, 3, 6, seed=0), "wlan": lambda: wlan_H,
         "reg39": lambda: codes.regular_code(900, 3, 9, seed=0)}[name]()
    g = graph.build_graph(H)
    G = eng.Graph(g, DEV)
    q = UniformQuantizer(sigma2_from_ebn0(1.0, g.R_c), 16)
    tb = tables.llr_tables(q.output_LLRs, g.d_c_max, g.d_v_max, 11)
    ch = q.sample_all_zero(g.n_v, 4100, np.random.default_rng(4)).astype(np.int32)
    ref = oracle.ib_decode(g, tb, ch, match=True, early_stop=False)
    for mode in ("1", "0"):
        for ncw in ("8", "4"):
            monkeypatch.setenv("IBL_FUSED_DBUF", mode)
            monkeypatch.setenv("IBL_FUSED_NCW", ncw)
            fo, _, fdec = _run(eng, g, tb, ch, True, False, graph_obj=G, path="fused")
            assert fdec.fused
            np.testing.assert_array_equal(fo, ref, err_msg=f"IBL_FUSED_DBUF={mode} IBL_FUSED_NCW={ncw}")


def test_ib_fused_path_selection(eng, wlan_H, dvb_H):
    g = graph.build_graph(wlan_H)
    G = eng.Graph(g, DEV)
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, 5)
    assert eng.IBDecoder(G, tb, True, 64).fused
    assert not eng.IBDecoder(G, tb, True, 64, path="passes").fused
    assert not eng.IBDecoder(G, tb, True, 64, force_generic=True).fused
    D = eng.Graph(graph.build_graph(dvb_H), DEV)
    tbd = tables.random_tables(16, 16, 7, 8, 5)
    assert not eng.IBDecoder(D, tbd, True, 64).fused         # E * 4 B = 907 KB of messages
    from informationbottleneckdecodingldpc_amd._lib import IBLError
    with pytest.raises(IBLError):
        eng.IBDecoder(D, tbd, True, 64, path="fused")


@pytest.mark.parametrize("n,fits", [(800, True), (1000, False)])
def test_ib_fused_limit_three_quads(eng, n, fits):
    """with the quad layout an odd quad count takes a whole 64-KiB super-region. A regular (9,12)
    code without matching needs 10 check tables / 9 decision tables a pass = 3 quads = 128 KiB + 3 KiB of raw
    images, so the fused kernel takes it up to E * 4 <= 29,680 B (ibldpc.h): N = 800 (E = 7,200) is fused, N = 1000
    (E = 9,000; fused under the round-4 layout's 96 KiB) runs the per-pass fast path. Both equal the oracle."""
    g = graph.build_graph(codes.regular_code(n, 9, 12, seed=2))
    assert g.d_c_max == 12 and g.d_v_max == 9 and g.n_e == 9 * n
    G = eng.Graph(g, DEV)
    imax, B = 5, 40
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, imax, seed=n)
    ch = np.random.default_rng(n).integers(0, 16, (g.n_v, B)).astype(np.int32)
    ref = oracle.ib_decode(g, tb, ch, match=False)
    out, _, dec = _run(eng, g, tb, ch, False, False, graph_obj=G)
    assert dec.fast_path and dec.fused == fits
    np.testing.assert_array_equal(out, ref)
    if not fits:
        from informationbottleneckdecodingldpc_amd._lib import IBLError
        with pytest.raises(IBLError):
            eng.IBDecoder(G, tb, False, B, path="fused")


def test_ib_early_stop_converging(eng, wlan_H):
    """LLR-quantised tables at good SNR: the batch converges before imax; same stop iteration and
    outputs as the oracle, with matching on."""
    g = graph.build_graph(wlan_H)
    q = UniformQuantizer(sigma2_from_ebn0(4.0, g.R_c), 16)
    imax = 30
    tb = tables.llr_tables(q.output_LLRs, g.d_c_max, g.d_v_max, imax)
    ch = q.sample_all_zero(g.n_v, 40, np.random.default_rng(3))
    ref, ref_it = oracle.ib_decode(g, tb, ch, match=True, early_stop=True, return_iters=True)
    out, it, _ = _run(eng, g, tb, ch, True, True)
    assert ref_it < imax - 1
    assert it == ref_it
    np.testing.assert_array_equal(out, ref)


def test_reference_golden_decode_on_host(golden, reg_H, wlan_H):
    """Drop-in decode_on_host (HIP kernels) == the reference's decode_on_host outputs."""
    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder import Discrete_LDPC_Decoder_class
    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import \
        Discrete_LDPC_Decoder_class_irregular
    z = golden
    for imax in (1, 2, 10):
        dec = Discrete_LDPC_Decoder_class(reg_H, imax, 16, 16, z[f"reg_imax{imax}_cn"], z[f"reg_imax{imax}_vn"], 4)
        for k in range(3):
            out = dec.decode_on_host(z[f"reg_imax{imax}_ch"][:, k])
            np.testing.assert_array_equal(out, z[f"reg_imax{imax}_out"][:, k])
        deci = Discrete_LDPC_Decoder_class_irregular(wlan_H, imax, 16, 16, z[f"wlan_imax{imax}_cn"],
                                                     z[f"wlan_imax{imax}_vn"], None, None, 4, match="true")
        for k in range(3):
            out = deci.decode_on_host(z[f"wlan_imax{imax}_ch"][:, k])
            np.testing.assert_array_equal(out, z[f"wlan_imax{imax}_out"][:, k].astype(np.float64))


def test_dropin_decode_opencl_and_errors(wlan_H):
    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import \
        Discrete_LDPC_Decoder_class_irregular
    g = graph.build_graph(wlan_H)
    imax = 8
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, imax, seed=11)
    B = 100
    dec = Discrete_LDPC_Decoder_class_irregular(wlan_H, imax, 16, 16, tb.cn, tb.vn, tb.match_cn, tb.match_vn, B,
                                                match="true")
    dec.init_OpenCL_decoding(B, 0)
    ch = np.random.default_rng(0).integers(0, 16, (g.n_v, B)).astype(np.int32)
    host_out = dec.decode_OpenCL(ch)                       # numpy in, numpy out
    ref = oracle.ib_decode(g, tb, ch, match=True, early_stop=True)
    np.testing.assert_array_equal(host_out, ref)
    buf = dec.decode_OpenCL(torch.from_numpy(ch).to(DEV), buffer_in=True, return_buffer=True)
    assert isinstance(buf, torch.Tensor) and buf.device.type == "cuda"
    np.testing.assert_array_equal(buf.cpu().numpy(), ref)
    assert dec.return_errors_all_zero(buf) == int((ref[:dec.data_len] < 8).sum())
    assert dec.data_len == 648


def test_full_size_dvbs2_properties(eng, dvb_H):
    """BASELINE size (DVB-S2 N=64800, B=8192, imax=50, match on): deterministic, shard-equivalent
    (1 batch == 2 half batches), and spot columns equal the oracle."""
    g = graph.build_graph(dvb_H)
    imax, B = 50, 8192
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, imax, seed=2)
    G = eng.Graph(g, DEV)
    dec = eng.IBDecoder(G, tb, True, B)
    assert dec.fast_path
    gen = torch.Generator(device=DEV)
    gen.manual_seed(0)
    ch = torch.randint(0, 16, (g.n_v, B), device=DEV, dtype=torch.uint8, generator=gen)
    o1 = dec.decode(ch, out_dtype=torch.uint8, early_stop=False).clone()
    o2 = dec.decode(ch, out_dtype=torch.uint8, early_stop=False).clone()
    assert torch.equal(o1, o2)
    h1 = dec.decode(ch[:, :B // 2].contiguous(), out_dtype=torch.uint8, early_stop=False).clone()
    h2 = dec.decode(ch[:, B // 2:].contiguous(), out_dtype=torch.uint8, early_stop=False).clone()
    assert torch.equal(torch.cat([h1, h2], 1), o1)
    # 64 columns spread over the batch (every row segment / chunk position class) against the oracle
    cols = sorted(set([0, 1, 511, 512, 1023, 1024, 4095, 8191] +
                      list(np.random.default_rng(5).choice(B, 56, replace=False))))
    assert len(cols) >= 64
    ref = oracle.ib_decode(g, tb, ch[:, cols].cpu().numpy().astype(np.int32), match=True)
    np.testing.assert_array_equal(o1[:, cols].cpu().numpy().astype(np.int32), ref)


def test_full_size_dvbs2_early_stop_converging(eng, dvb_H):
    """BASELINE size (DVB-S2, B=8192, i_max=50) with early stop ON and a batch that converges.

    The stop is batch-global (discrete_LDPC_decoder_irreg.py:310-320: the summed syndrome of the
    variable-to-check messages of the WHOLE batch must be zero); with random noise one of 8192
    codewords whose messages keep oscillating is enough to prevent it (tools/diag_early_stop.py: no
    stop at 2.5-5 dB for B=8192, the oracle agrees on small batches). So the batch is 16 copies of a
    512-codeword sample that converges (LLR tables, 5 dB, the degree-1 parity bit's channel value set
    reliable — it is forwarded unchanged, kernels_template_irreg.cl:131-136): the 8192-column decode
    must stop at the same L as the 512-column one, every copy must decode identically, and 64
    columns must equal the oracle run for exactly L iterations."""
    g = graph.build_graph(dvb_H)
    q = UniformQuantizer(sigma2_from_ebn0(5.0, g.R_c), 16)
    imax, B, S = 50, 8192, 512
    tb = tables.llr_tables(q.output_LLRs, g.d_c_max, g.d_v_max, imax)
    G = eng.Graph(g, DEV)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(7)
    base = q.sample_all_zero_device(g.n_v, S, DEV, generator=gen)
    base[np.flatnonzero(g.vn_deg == 1)] = 15
    it = torch.zeros(1, dtype=torch.int32, device=DEV)
    small = eng.IBDecoder(G, tb, True, S).decode(base, out_dtype=torch.uint8, early_stop=True, iters=it).clone()
    L_small = int(it.item())
    assert 1 <= L_small < imax - 1, L_small
    ch = base.repeat(1, B // S).contiguous()
    out = eng.IBDecoder(G, tb, True, B).decode(ch, out_dtype=torch.uint8, early_stop=True, iters=it)
    L = int(it.item())
    assert L == L_small
    assert torch.equal(out, small.repeat(1, B // S))
    assert int(eng.count_below(out, g.n_v, 8).item()) == 0
    cols = sorted(np.random.default_rng(6).choice(B, 64, replace=False))
    x = ch[:, cols].cpu().numpy().astype(np.int32)
    tbL = tables.llr_tables(q.output_LLRs, g.d_c_max, g.d_v_max, L + 1)
    np.testing.assert_array_equal(tbL.cn, tb.cn[:tbL.cn.size])      # same per-iteration tables
    np.testing.assert_array_equal(tbL.vn, tb.vn[:tbL.vn.size])
    ref = oracle.ib_decode(g, tbL, x, match=True, early_stop=False)
    np.testing.assert_array_equal(out[:, cols].cpu().numpy().astype(np.int32), ref)
    _, it64 = oracle.ib_decode(g, tb, x, match=True, early_stop=True, return_iters=True)
    assert it64 <= L


def test_full_size_dvbs2_decodes_all_zero(eng, dvb_H):
    """LLR-quantised tables at 3 dB: every one of 8192 all-zero codewords decodes (0 errors).
    (No early stop happens here: the degree-1 parity bit forwards its channel value unchanged,
    kernels_template_irreg.cl:131-136, so ~8 % of codewords keep one unsatisfied check and the
    batch-global syndrome never reaches zero.)"""
    g = graph.build_graph(dvb_H)
    q = UniformQuantizer(sigma2_from_ebn0(3.0, g.R_c), 16)
    imax, B = 50, 8192
    tb = tables.llr_tables(q.output_LLRs, g.d_c_max, g.d_v_max, imax)
    dec = eng.IBDecoder(eng.Graph(g, DEV), tb, True, B)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(1)
    ch = q.sample_all_zero_device(g.n_v, B, DEV, generator=gen)
    it = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = dec.decode(ch, out_dtype=torch.uint8, early_stop=True, iters=it)
    errs = int(eng.count_below(out, g.data_len, 8).item())
    assert errs == 0


def test_fused_lds_cap_survives_a_smaller_decoder(wlan_H):
    """The fused kernel's dynamic-LDS cap belongs to the kernel instantiation: a large-LDS decoder (regular
    (3,6) N=8000 with two table sets) created first, then a smaller one (WLAN) on the same instantiation, and
    the first decodes again — bit-exact against the oracle."""
    from informationbottleneckdecodingldpc_amd import codes, engine
    g1 = graph.build_graph(codes.regular_code(8000, 3, 6, seed=0))
    tb1 = tables.random_tables(16, 16, g1.d_c_max, g1.d_v_max, 6, seed=4)
    big = engine.IBDecoder(engine.Graph(g1, DEV), tb1, False, 64, path="fused")
    g2 = graph.build_graph(wlan_H)
    tb2 = tables.random_tables(16, 16, g2.d_c_max, g2.d_v_max, 6, seed=5)
    small = engine.IBDecoder(engine.Graph(g2, DEV), tb2, False, 64, path="fused")
    x2 = np.random.default_rng(2).integers(0, 16, (g2.n_v, 64)).astype(np.int32)
    o2 = small.decode(torch.from_numpy(x2).to(DEV), early_stop=False).cpu().numpy()
    np.testing.assert_array_equal(o2, oracle.ib_decode(g2, tb2, x2, match=False))
    x1 = np.random.default_rng(1).integers(0, 16, (g1.n_v, 64)).astype(np.int32)
    o1 = big.decode(torch.from_numpy(x1).to(DEV), early_stop=False).cpu().numpy()
    np.testing.assert_array_equal(o1, oracle.ib_decode(g1, tb1, x1, match=False))


def test_u8_staging_quad_words(eng, wlan_H):
    """The u8 channel staging's 16-byte path (rows of 16-byte multiples: whole 1024-word items; the rest of a row
    and other rows by words) decodes what the int32 staging decodes: B = 8208 = one whole item + 2 words per row,
    a 16-byte aligned base and one at +16 (the view's rows still 16-byte multiples), per-pass kernels."""
    g = graph.build_graph(wlan_H)
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, 3, seed=9)
    B = 8208
    x = torch.from_numpy(np.random.default_rng(7).integers(0, 16, (g.n_v, B)).astype(np.uint8)).to(DEV)
    dec = eng.IBDecoder(eng.Graph(g, DEV), tb, True, B, path="passes")
    ref = dec.decode(x.to(torch.int32), out_dtype=torch.uint8, early_stop=False).clone()
    np.testing.assert_array_equal(ref[:, :3].cpu().numpy(), oracle.ib_decode(g, tb, x[:, :3].cpu().numpy(), match=True))
    out = dec.decode(x, out_dtype=torch.uint8, early_stop=False)
    assert torch.equal(out, ref)
    buf = torch.zeros(g.n_v * B + 16, dtype=torch.uint8, device=DEV)
    xv = buf[16:].view(g.n_v, B)
    xv.copy_(x)
    assert torch.equal(dec.decode(xv, out_dtype=torch.uint8, early_stop=False), ref)


@pytest.mark.parametrize("path", ["fused", "passes"])
def test_misaligned_u8_channel(eng, wlan_H, path):
    """A contiguous u8 channel view at an odd byte offset (B % 4 == 0, so the staging kernels' dword path
    would apply to an aligned pointer) decodes bit-exactly: the dword loads are taken only when aligned."""
    g = graph.build_graph(wlan_H)
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, 5, seed=8)
    B = 64
    x = np.random.default_rng(6).integers(0, 16, (g.n_v, B)).astype(np.uint8)
    buf = torch.zeros(g.n_v * B + 1, dtype=torch.uint8, device=DEV)
    ch = buf[1:].view(g.n_v, B)
    ch.copy_(torch.from_numpy(x).to(DEV))
    assert ch.is_contiguous() and ch.data_ptr() % 4 == 1
    dec = eng.IBDecoder(eng.Graph(g, DEV), tb, True, B, path=path)
    out = dec.decode(ch, early_stop=False).cpu().numpy()
    np.testing.assert_array_equal(out, oracle.ib_decode(g, tb, x, match=True))


