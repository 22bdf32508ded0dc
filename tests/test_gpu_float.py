"""GPU parity of the float min-sum / BP decoders against the CPU oracles (restatements of
kernels_min_and_BP.cl in fp64 and, for min-sum, fp32; the reference's own float host path is
broken, SURVEY Appendix C3, so parity is pinned by the kernel text).

Bars (written in the tests):
  * fp64 min-sum: bit-identical APP LLRs and stop iteration (vs the fp64 oracle);
  * fp64 BP: |x-y| <= 1e-9 (device exp/log vs glibc differ in the last ulps);
  * fp32 min-sum (BASELINE C3's build): bit-identical APP LLRs and stop iteration vs the fp32
    oracle — the same selections and ordered adds in IEEE single — at every i_max, including C3's
    N=1944 / i_max=50, on the per-pass and the fused path;
  * fp32 min-sum vs the fp64 reference precision: the decoder's error statistic (paired per-codeword
    bit-error counts) within a stated confidence bound — unnormalised min-sum on the quantised LLR
    alphabet is chaotic once codewords fail to converge: sums that cancel exactly to 0 in fp64
    (sign() = 0 kills a message) come out as +-1 ulp in fp32 and the trajectories separate
    (tools/diag_float32.py);
  * fp32 BP vs the fp64 oracle: SURVEY H5's |x-y| <= 1e-5*max(|x|,|y|) + 1e-4 on every APP LLR of
    every codeword the fp64 decoder converges on, identical stop iteration and identical hard
    decisions wherever the oracle's LLR lies outside that band around 0; on DVB-S2 (C5's code) up to
    i_max = 100 this holds for every codeword (measured: max |x-y| 4e-4).
"""
import numpy as np
import pytest
import torch

from informationbottleneckdecodingldpc_amd import codes, graph
from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0
from oracle import oracle
from tests._codes import mixed_code

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
REL = 1e-5
TOL_ABS = 1e-4                    # |x-y| <= 1e-5*max(|x|,|y|) + 1e-4


@pytest.fixture(scope="module")
def eng():
    from informationbottleneckdecodingldpc_amd import engine
    return engine


def _llrs(g, B, ebn0, seed, quantised=True):
    q = UniformQuantizer(sigma2_from_ebn0(ebn0, g.R_c), 16)
    rng = np.random.default_rng(seed)
    if quantised:   # the reference's "quantised BP" input (quantize_direct_OpenCL_LLR)
        return q.llr_of(q.sample_all_zero(g.n_v, B, rng))
    y = 1.0 + np.sqrt(q.sigma_n2) * rng.standard_normal((g.n_v, B))
    return 2 * y / q.sigma_n2


def _gpu(eng, g, kind, imax, llr, prec, early, graph_obj=None, path="auto"):
    G = graph_obj or eng.Graph(g, DEV)
    dec = eng.FloatDecoder(G, kind, imax, llr.shape[1], precision=prec, path=path)
    it = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = dec.decode(torch.from_numpy(llr).to(DEV).to(prec), early_stop=early, iters=it)
    torch.cuda.synchronize()
    return out.double().cpu().numpy(), int(it.item())


@pytest.mark.parametrize("kind", [oracle.MINSUM, oracle.BP])
@pytest.mark.parametrize("name,imax,B,early,ebn0", [("wlan", 2, 3, False, 1.0), ("wlan", 10, 300, False, 1.5),
                                                     ("wlan", 20, 129, True, 4.0), ("reg", 8, 64, False, 2.0),
                                                     ("dvb", 5, 4, False, 1.0)])
@pytest.mark.parametrize("path", ["auto", "passes"])
def test_float64_vs_oracle(eng, kind, name, imax, B, early, ebn0, path, wlan_H, reg_H, dvb_H):
    g = graph.build_graph({"wlan": wlan_H, "reg": reg_H, "dvb": dvb_H}[name])
    llr = _llrs(g, B, ebn0, seed=imax + B, quantised=(kind == oracle.BP))
    ref, ref_it = oracle.float_decode(g, kind, imax, llr, early_stop=early, return_iters=True)
    out, it = _gpu(eng, g, kind, imax, llr, torch.float64, early, path=path)
    assert it == ref_it
    if kind == oracle.MINSUM:
        np.testing.assert_array_equal(out, ref)
    else:
        np.testing.assert_allclose(out, ref, rtol=0, atol=1e-9)


def _h5(out, ref):
    """Entries outside SURVEY H5's tolerance."""
    return np.abs(out - ref) > REL * np.maximum(np.abs(out), np.abs(ref)) + TOL_ABS


def _hard_flips(out, ref):
    """Hard-decision differences where the oracle's LLR lies outside the tolerance band around 0 (a
    value within the band may take either sign and still meet H5)."""
    return int((((out < 0) != (ref < 0)) & (np.abs(ref) > REL * np.abs(ref) + TOL_ABS)).sum())


def _code_of(name, wlan_H, reg_H, dvb_H):
    from informationbottleneckdecodingldpc_amd import codes
    if name == "wlan1944":
        return codes.wlan_80211n(81)
    return {"wlan": wlan_H, "reg": reg_H, "dvb": dvb_H}[name]


@pytest.mark.parametrize("name,imax,B,early,ebn0", [
    ("wlan1944", 50, 256, False, 1.0),    # BASELINE C3: N=1944, i_max=50 (non-converging batch)
    ("wlan1944", 50, 300, True, 3.0),     # C3 code, early stop requested
    ("wlan1944", 30, 64, True, 4.5),      # batch converges: stop before imax-1
    ("wlan", 50, 129, True, 2.0),
    ("reg", 50, 70, False, 2.0),
    ("dvb", 50, 8, False, 1.0)])
@pytest.mark.parametrize("path", ["auto", "passes"])
def test_float32_minsum_bit_exact(eng, name, imax, B, early, ebn0, path, wlan_H, reg_H, dvb_H):
    """fp32 min-sum == the fp32 oracle bit for bit (selections + ordered IEEE single adds)."""
    g = graph.build_graph(_code_of(name, wlan_H, reg_H, dvb_H))
    llr = _llrs(g, B, ebn0, seed=5 * imax + B).astype(np.float32)
    ref, ref_it = oracle.float32_decode(g, imax, llr, early_stop=early, return_iters=True)
    out, it = _gpu(eng, g, oracle.MINSUM, imax, llr, torch.float32, early, path=path)
    assert it == ref_it
    np.testing.assert_array_equal(out, ref.astype(np.float64))


@pytest.mark.parametrize("ebn0", [1.0, 2.0, 3.0])
def test_float32_minsum_c3_error_statistics(eng, ebn0):
    """BASELINE C3 (WLAN N=1944 min-sum fp32, i_max=50) vs the reference's fp64 precision on the same
    channel: the per-codeword bit-error counts d_c = e32_c - e64_c are paired; |mean(d)| must lie
    within 4 standard errors (two-sided, ~6e-5 false-alarm rate under 'same decoder statistic'), and
    so must the discordant frame errors (McNemar: |n10 - n01| <= 4 sqrt(n10 + n01))."""
    from informationbottleneckdecodingldpc_amd import codes
    g = graph.build_graph(codes.wlan_80211n(81))
    B = 512
    llr = _llrs(g, B, ebn0, seed=int(ebn0 * 10))
    ref = oracle.float_decode(g, oracle.MINSUM, 50, llr)
    out, _ = _gpu(eng, g, oracle.MINSUM, 50, llr.astype(np.float32), torch.float32, False)
    e64 = (ref[:g.data_len] < 0).sum(0).astype(np.float64)
    e32 = (out[:g.data_len] < 0).sum(0).astype(np.float64)
    d = e32 - e64
    se = d.std(ddof=1) / np.sqrt(B) if B > 1 else 0.0
    assert abs(d.mean()) <= 4 * se, (d.mean(), se, e32.sum(), e64.sum())
    n10 = int(((e32 > 0) & (e64 == 0)).sum())
    n01 = int(((e32 == 0) & (e64 > 0)).sum())
    assert abs(n10 - n01) <= 4 * np.sqrt(n10 + n01), (n10, n01)


@pytest.mark.parametrize("name,imax,B,ebn0", [
    ("wlan", 10, 256, 1.5), ("wlan", 20, 100, 2.0), ("reg", 20, 70, 2.0), ("dvb", 10, 8, 1.2)])
def test_float32_bp_vs_oracle(eng, name, imax, B, ebn0, wlan_H, reg_H, dvb_H):
    g = graph.build_graph(_code_of(name, wlan_H, reg_H, dvb_H))
    llr = _llrs(g, B, ebn0, seed=3 * imax + B, quantised=True)
    ref = oracle.float_decode(g, oracle.BP, imax, llr)
    out, _ = _gpu(eng, g, oracle.BP, imax, llr, torch.float32, False)
    bad = _h5(out, ref)
    assert bad.sum() == 0, f"{bad.sum()} of {bad.size} LLRs outside H5, max |x-y| {np.abs(out - ref).max():.3e}"
    assert _hard_flips(out, ref) == 0


@pytest.mark.parametrize("ebn0,early", [(0.6, False), (1.0, True), (1.5, False)])
def test_float32_bp_c5_dvbs2_imax100(eng, dvb_H, ebn0, early):
    """BASELINE C5 (DVB-S2 BP fp32, i_max=100) on a small batch vs the fp64 oracle: every APP LLR
    within H5, identical hard decisions and stop iteration (the fp32 forward-backward check node)."""
    g = graph.build_graph(dvb_H)
    llr = _llrs(g, 6, ebn0, seed=int(ebn0 * 100))
    ref, ref_it = oracle.float_decode(g, oracle.BP, 100, llr, early_stop=early, return_iters=True)
    out, it = _gpu(eng, g, oracle.BP, 100, llr, torch.float32, early)
    assert it == ref_it
    bad = _h5(out, ref)
    assert bad.sum() == 0, f"{bad.sum()} of {bad.size} LLRs outside H5, max |x-y| {np.abs(out - ref).max():.3e}"
    assert _hard_flips(out, ref) == 0


def test_float32_bp_wlan1944_converged_codewords(eng):
    """WLAN N=1944 BP fp32 at i_max=50/100: H5 on every codeword the fp64 decoder converges on (zero
    decided errors for the all-zero word); codewords stuck in a trapping set oscillate and their fp32
    and fp64 trajectories separate, so for them only the decided-error total is compared."""
    from informationbottleneckdecodingldpc_amd import codes
    g = graph.build_graph(codes.wlan_80211n(81))
    for imax, ebn0 in ((50, 1.5), (100, 2.0)):
        llr = _llrs(g, 32, ebn0, seed=imax)
        ref = oracle.float_decode(g, oracle.BP, imax, llr)
        out, _ = _gpu(eng, g, oracle.BP, imax, llr, torch.float32, False)
        conv = (ref < 0).sum(0) == 0
        assert conv.sum() >= 24, conv.sum()
        bad = _h5(out[:, conv], ref[:, conv])
        assert bad.sum() == 0, f"{bad.sum()} LLRs of converged codewords outside H5"
        assert ((out[:, conv] < 0).sum() == 0)
        e_ref, e_gpu = int((ref[:, ~conv] < 0).sum()), int((out[:, ~conv] < 0).sum())
        assert abs(e_gpu - e_ref) <= max(10, 4 * np.sqrt(e_ref + 1)), (e_gpu, e_ref)


@pytest.mark.parametrize("kind", [oracle.MINSUM, oracle.BP])
@pytest.mark.parametrize("path", ["auto", "passes"])
def test_float_mixed_degrees(eng, kind, path):
    """Every float node body: check degrees 2..16 (incl. degree 2's empty folds and the > 8 immediate-
    store / MAXD=16 instantiations), variable degrees 1..16; fp64 against the fp64 oracle (min-sum
    bit-exact, BP 1e-9), fp32 min-sum bit-exact against the fp32 oracle, fp32 BP within H5."""
    g = graph.build_graph(mixed_code(np.arange(2, 17), np.arange(1, 17), 600, seed=15))
    assert g.d_c_max == 16 and g.d_v_max == 16
    imax, B = 6, 260
    llr = _llrs(g, B, 2.0, seed=kind + 11)
    G = eng.Graph(g, DEV)
    ref, ref_it = oracle.float_decode(g, kind, imax, llr, early_stop=True, return_iters=True)
    out, it = _gpu(eng, g, kind, imax, llr, torch.float64, True, graph_obj=G, path=path)
    assert it == ref_it
    if kind == oracle.MINSUM:
        np.testing.assert_array_equal(out, ref)
        r32 = oracle.float32_decode(g, imax, llr.astype(np.float32)).astype(np.float64)
        o32, _ = _gpu(eng, g, kind, imax, llr.astype(np.float32), torch.float32, False, graph_obj=G, path=path)
        np.testing.assert_array_equal(o32, r32)
    else:
        np.testing.assert_allclose(out, ref, rtol=0, atol=1e-9)
        ref_f = oracle.float_decode(g, kind, imax, llr)
        o32, _ = _gpu(eng, g, kind, imax, llr, torch.float32, False, graph_obj=G, path=path)
        assert _h5(o32, ref_f).sum() == 0
        assert _hard_flips(o32, ref_f) == 0


def test_imax1_outputs_channel(eng, wlan_H):
    g = graph.build_graph(wlan_H)
    llr = _llrs(g, 5, 1.0, 0)
    ref = oracle.float_decode(g, oracle.MINSUM, 1, llr)
    out, it = _gpu(eng, g, oracle.MINSUM, 1, llr, torch.float64, True)
    assert it == 0
    np.testing.assert_array_equal(out, ref)
    np.testing.assert_array_equal(out, llr)


def test_dropin_min_sum_and_bp(wlan_H):
    from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular
    from informationbottleneckdecodingldpc_amd.min_sum_decoder_irreg import Min_Sum_Decoder_class_irregular
    g = graph.build_graph(wlan_H)
    llr = _llrs(g, 50, 1.5, 9)
    ms = Min_Sum_Decoder_class_irregular(wlan_H, 20, 16, 50, precision=torch.float64)
    ms.init_OpenCL_decoding(50)
    out = ms.decode_OpenCL_min_sum(llr)
    ref = oracle.float_decode(g, oracle.MINSUM, 20, llr, early_stop=True)
    np.testing.assert_array_equal(out, ref)
    buf = ms.decode_OpenCL_min_sum(torch.from_numpy(llr).to(DEV), buffer_in=True, return_buffer=True)
    assert ms.return_errors_all_zero(buf) == float((ref[:ms.data_len] < 0).sum())
    bp = BeliefPropagationDecoderClassIrregular(wlan_H, 20, 16, 50)
    bp.init_OpenCL_decoding(50)
    out = bp.decode_OpenCL_belief_propagation(llr)
    assert out.dtype == np.float32 and out.shape == llr.shape
    hd = bp.decode_on_host(llr[:, 0])
    assert hd.shape == (g.n_v,)


@pytest.mark.parametrize("prec", [torch.float64, torch.float32])
@pytest.mark.parametrize("ebn0", [0.8, 1.4])
def test_dropin_bp_c5_vs_oracle(dvb_H, prec, ebn0):
    """The reference-named BP class on C5's code (DVB-S2, i_max=100), as the BP BER driver calls it
    (WLAN/BER_simulation_OpenCL_quant_BP.py:105-110: decode_OpenCL_belief_propagation with early stop,
    then return_errors_all_zero): APP LLRs vs the fp64 oracle (fp64 build 1e-9, fp32 build SURVEY H5 with
    no hard flips) and the error count equal to the oracle's (bp_decoder_irreg.py:221-295)."""
    from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular
    g = graph.build_graph(dvb_H)
    B = 8
    llr = _llrs(g, B, ebn0, seed=int(ebn0 * 10) + 3)
    if prec == torch.float32:
        llr = llr.astype(np.float32).astype(np.float64)     # the fp32 build's inputs, exactly
    bp = BeliefPropagationDecoderClassIrregular(dvb_H, 100, 16, B, precision=prec)
    assert bp.data_len == 32399                             # reference R_c quirk
    bp.init_OpenCL_decoding(B)
    ref = oracle.float_decode(g, oracle.BP, 100, llr, early_stop=True)
    buf = bp.decode_OpenCL_belief_propagation(torch.from_numpy(llr).to(DEV).to(prec), buffer_in=True,
                                              return_buffer=True)
    assert buf.dtype == prec and tuple(buf.shape) == llr.shape
    out = buf.double().cpu().numpy()
    if prec == torch.float64:
        np.testing.assert_allclose(out, ref, rtol=0, atol=1e-9)
    else:
        bad = _h5(out, ref)
        assert bad.sum() == 0, f"{bad.sum()} LLRs outside H5, max |x-y| {np.abs(out - ref).max():.3e}"
        assert _hard_flips(out, ref) == 0
    assert bp.return_errors_all_zero(buf) == float((ref[:bp.data_len] < 0).sum())
    host = bp.decode_OpenCL_belief_propagation(llr)         # host ndarray in and out
    np.testing.assert_array_equal(host.astype(np.float64), out)


def test_count_below_matches_numpy(eng):
    x = torch.randn(513, 77, device=DEV)
    assert int(eng.count_below(x, 300, 0.0).item()) == int((x[:300] < 0).sum().item())
    y = torch.randint(0, 16, (100, 33), device=DEV, dtype=torch.int32)
    assert int(eng.count_below(y, 100, 8).item()) == int((y < 8).sum().item())


# ------------------------------------------------------------------ fused on-chip path
# The fused kernel (fl_fused: a workgroup keeps 4 fp32 / 2 fp64 codewords in LDS for all
# iterations) runs the per-pass kernels' node bodies in the same order, so its outputs and stop
# iterations must equal the per-pass path's bit for bit, in both precisions and for BP as well.
@pytest.mark.parametrize("prec", [torch.float32, torch.float64])
@pytest.mark.parametrize("kind", [oracle.MINSUM, oracle.BP])
@pytest.mark.parametrize("name,imax,B,early,ebn0", [
    ("wlan", 10, 301, False, 1.5),     # ragged last group
    ("wlan", 30, 257, True, 1.0),      # early stop requested, batch never satisfied: one pass
    ("wlan", 30, 64, True, 4.0),       # batch-global stop before imax-1: pass 2 re-runs to L
    ("wlan", 2, 5, True, 1.0),
    ("reg", 12, 130, True, 3.0),
    ("wlan1944", 8, 1000, False, 1.5)])
def test_fused_equals_passes(eng, prec, kind, name, imax, B, early, ebn0, wlan_H, reg_H):
    from informationbottleneckdecodingldpc_amd import codes
    H = {"wlan": wlan_H, "reg": reg_H}.get(name)
    if H is None:
        H = codes.wlan_80211n(81)
    g = graph.build_graph(H)
    G = eng.Graph(g, DEV)
    llr = _llrs(g, B, ebn0, seed=imax * 7 + B, quantised=True)
    fused, it_f = _gpu(eng, g, kind, imax, llr, prec, early, graph_obj=G, path="fused")
    passes, it_p = _gpu(eng, g, kind, imax, llr, prec, early, graph_obj=G, path="passes")
    assert it_f == it_p
    np.testing.assert_array_equal(fused, passes)


@pytest.mark.parametrize("prec", [torch.float32, torch.float64])
@pytest.mark.parametrize("kind", [oracle.MINSUM, oracle.BP])
def test_fused_full_tasks_of_check_degree_above_8(eng, prec, kind):
    """A code with full (64-node) check tasks of degree 10 — the fused kernel's constant-stride body
    covers degrees <= 8 only, so these tasks must take the general body (they were skipped).
    Regular (3,10), N=960: 288 checks of degree 10 = 4 full tasks + one of 32. Fused == per-pass, and the
    fp64 min-sum decode == the oracle."""
    g = graph.build_graph(codes.regular_code(960, 3, 10, seed=3))
    assert g.d_c_max == 10 and g.n_c >= 256
    G = eng.Graph(g, DEV)
    B, imax = 70, 12
    llr = _llrs(g, B, 3.0, seed=41, quantised=True)
    fused, it_f = _gpu(eng, g, kind, imax, llr, prec, True, graph_obj=G, path="fused")
    passes, it_p = _gpu(eng, g, kind, imax, llr, prec, True, graph_obj=G, path="passes")
    assert it_f == it_p
    np.testing.assert_array_equal(fused, passes)
    if kind == oracle.MINSUM and prec == torch.float64:
        ref, ref_it = oracle.float_decode(g, kind, imax, llr, early_stop=True, return_iters=True)
        assert it_f == ref_it
        np.testing.assert_array_equal(fused, ref)


def test_fused_stop_iteration_and_outputs_vs_oracle(eng, wlan_H):
    """Early stop inside the fused path (pass 2) against the fp64 oracle directly."""
    g = graph.build_graph(wlan_H)
    llr = _llrs(g, 40, 3.5, seed=5)
    ref, ref_it = oracle.float_decode(g, oracle.MINSUM, 25, llr, early_stop=True, return_iters=True)
    assert 1 <= ref_it < 24, ref_it
    out, it = _gpu(eng, g, oracle.MINSUM, 25, llr, torch.float64, True, path="fused")
    assert it == ref_it
    np.testing.assert_array_equal(out, ref)


def test_fused_path_selection(eng, wlan_H, dvb_H):
    G = eng.Graph(graph.build_graph(wlan_H), DEV)
    assert eng.FloatDecoder(G, 0, 5, 16).fused
    assert not eng.FloatDecoder(G, 0, 5, 16, path="passes").fused
    D = eng.Graph(graph.build_graph(dvb_H), DEV)
    assert not eng.FloatDecoder(D, 0, 5, 16).fused       # (E + N) * 16 B = 4.7 MB > 160 KiB
    from informationbottleneckdecodingldpc_amd._lib import IBLError
    with pytest.raises(IBLError):
        eng.FloatDecoder(D, 0, 5, 16, path="fused")
    # the fused kernel keeps the variable-edge slot indices in LDS too (u16, task rows padded to 64):
    # regular (3,6) N=2304: 64 N + 16 + 6 N = 161,296 B fits; N=2400: the messages alone (153,616 B) would,
    # with the indices (168,016 B) they do not -> the per-pass path
    for n, fits in ((2304, True), (2400, False)):
        R = eng.Graph(graph.build_graph(codes.regular_code(n, 3, 6, seed=1)), DEV)
        assert eng.FloatDecoder(R, 0, 5, 16).fused == fits
        if not fits:
            with pytest.raises(IBLError):
                eng.FloatDecoder(R, 0, 5, 16, path="fused")


@pytest.mark.parametrize("path", ["auto", "passes"])
def test_float32_minsum_tiny_llrs(eng, wlan_H, path):
    """The closed-form min-sum check node (float_kernels.hip fl_cn_body) equals the reference fold
    t = sgn(m t) min(|t|, |m|) as long as no product m t underflows; scaling the quantised LLRs by 2^-50 (the
    boundary stated there: every nonzero message stays a multiple of the smallest LLR's ulp, so products stay
    >= 2^-146) keeps the fp32 GPU decode bit-exact with the literal fp32 oracle fold."""
    g = graph.build_graph(wlan_H)
    llr = _llrs(g, 64, 1.5, seed=17).astype(np.float32)
    mn = float(np.abs(llr[llr != 0]).min())
    llr = llr * np.float32(2.0 ** (-50 - int(np.floor(np.log2(mn)))))      # exact power-of-two scaling
    assert 2.0 ** -50 <= np.abs(llr[llr != 0]).min() < 2.0 ** -49
    ref = oracle.float32_decode(g, 20, llr)
    out, _ = _gpu(eng, g, oracle.MINSUM, 20, llr, torch.float32, False, path=path)
    np.testing.assert_array_equal(out, ref.astype(np.float64))


@pytest.mark.parametrize("prec,kind", [(torch.float32, oracle.MINSUM), (torch.float64, oracle.MINSUM)])
@pytest.mark.parametrize("path", ["auto", "passes"])
def test_float_infinite_channel_llrs(eng, wlan_H, prec, kind, path):
    """+-inf channel LLRs into min-sum (known bits; ibldpc.h's precondition allows them there): the
    variable messages clamp to +-llr_max and the APP LLR of such a bit is +-inf — as the oracle (the
    kernel text's clamp(ch + sum) and unclamped ch + sum) computes; fp32 and fp64 bit-exact. (BP is
    excluded by the precondition: the reference's box-plus log((1 + e^(a+b)) / (e^a + e^b)) is NaN for
    an infinite input and the clamp then returns -llr_max, kernels_min_and_BP.cl:5-9,69.)"""
    g = graph.build_graph(wlan_H)
    B = 96
    llr = _llrs(g, B, 1.5, seed=77)
    rng = np.random.default_rng(78)
    pos = rng.random(llr.shape) < 0.02
    llr[pos] = np.where(rng.random(pos.sum()) < 0.8, np.inf, -np.inf)
    if prec == torch.float32 and kind == oracle.MINSUM:
        llr = llr.astype(np.float32)
        ref = oracle.float32_decode(g, 20, llr).astype(np.float64)
    else:
        ref = oracle.float_decode(g, kind, 20, llr.astype(np.float32).astype(np.float64)
                                  if prec == torch.float32 else llr)
    out, _ = _gpu(eng, g, kind, 20, llr, prec, False, path=path)
    assert not np.isnan(out).any() and not np.isnan(ref).any()
    inf = np.isinf(ref)
    assert inf.sum() >= pos.sum() and np.array_equal(np.isinf(out), inf)
    np.testing.assert_array_equal(out[inf], ref[inf])
    if kind == oracle.MINSUM:
        np.testing.assert_array_equal(out, ref)
    elif prec == torch.float64:
        np.testing.assert_allclose(out[~inf], ref[~inf], rtol=0, atol=1e-9)
    else:
        assert _h5(out[~inf], ref[~inf]).sum() == 0


@pytest.mark.parametrize("ebn0", [2.5, 3.0])
def test_float32_minsum_c3_converged_codewords_h5(eng, ebn0):
    """BASELINE C3 (WLAN N=1944 min-sum, i_max=50) fp32 vs the reference's fp64 precision per LLR (north_star:
    "within 1e-5 relative"): on every codeword the fp64 decoder converges on (>= 75 % of the batch), every
    APP LLR within H5 (1e-5 max(|x|,|y|) + 1e-4) and identical hard decisions; codewords fp64 does not
    converge on are the chaotic regime of test_float32_minsum_c3_error_statistics. Same bar as the BP
    test_float32_bp_wlan1944_converged_codewords."""
    from informationbottleneckdecodingldpc_amd import codes
    g = graph.build_graph(codes.wlan_80211n(81))
    B = 256
    llr = _llrs(g, B, ebn0, seed=int(ebn0 * 100) + 1)
    ref = oracle.float_decode(g, oracle.MINSUM, 50, llr)
    out, _ = _gpu(eng, g, oracle.MINSUM, 50, llr.astype(np.float32), torch.float32, False)
    conv = (ref < 0).sum(0) == 0
    assert conv.sum() >= 0.75 * B, conv.sum()
    d = np.abs(out[:, conv] - ref[:, conv])
    rel = d / np.maximum(np.maximum(np.abs(out[:, conv]), np.abs(ref[:, conv])), 1e-30)
    print(f"C3 fp32 vs fp64 min-sum at {ebn0} dB: {int(conv.sum())}/{B} converged, max |x-y| {d.max():.3e}, "
          f"max rel {rel.max():.3e}")
    bad = _h5(out[:, conv], ref[:, conv])
    assert bad.sum() == 0, f"{bad.sum()} LLRs of converged codewords outside H5, max |x-y| {d.max():.3e}"
    assert ((out[:, conv] < 0) == (ref[:, conv] < 0)).all()


# ------------------------------------------------------------------ degree-2 variable fold (per-pass path)
@pytest.mark.parametrize("prec", [torch.float32, torch.float64])
@pytest.mark.parametrize("kind", [oracle.MINSUM, oracle.BP])
@pytest.mark.parametrize("name,imax,B,early,ebn0", [
    ("dvb", 12, 300, False, 1.0),     # C5's code: 32,399 degree-2 variables, every check folds two
    ("dvb", 30, 260, True, 2.0),      # early stop: folded passes write the variable inbox too (mode 2)
    ("dvb", 2, 7, False, 1.0),        # one check pass: it is the last, nothing folds
    ("wlan", 20, 257, True, 1.5)])    # dual-diagonal parity: degree-2 variables of the WLAN code
def test_float_fold_equals_unfolded(eng, prec, kind, name, imax, B, early, ebn0, wlan_H, dvb_H, monkeypatch):
    """The fold (the check pass computes a degree-2 variable's outgoing message, clamp(ch + m) in the
    variable pass's order, straight into the next check pass's inbox; the variable pass skips it) gives the
    same bits and stop iteration as the unfolded per-pass path (IBL_FL_FOLD=0), fp32 and fp64, min-sum and BP;
    fp64 min-sum also equals the oracle."""
    H = {"dvb": dvb_H, "wlan": wlan_H}[name]
    g = graph.build_graph(H)
    G = eng.Graph(g, DEV)
    llr = _llrs(g, B, ebn0, seed=imax * 3 + B, quantised=True)
    res = {}
    for fold in ("1", "0"):
        monkeypatch.setenv("IBL_FL_FOLD", fold)
        dec = eng.FloatDecoder(G, kind, imax, B, precision=prec, path="passes")
        n2 = int((np.asarray(g.vn_deg) == 2).sum())
        if fold == "1":
            assert dec.folded > 0 and dec.folded <= n2
            if name == "dvb":
                assert dec.folded == n2 == 32399
        else:
            assert dec.folded == 0
        it = torch.zeros(1, dtype=torch.int32, device=DEV)
        out = dec.decode(torch.from_numpy(llr).to(DEV).to(prec), early_stop=early, iters=it)
        res[fold] = (out.double().cpu().numpy(), int(it.item()))
    assert res["1"][1] == res["0"][1]
    np.testing.assert_array_equal(res["1"][0], res["0"][0])
    if kind == oracle.MINSUM and prec == torch.float64:
        ref, ref_it = oracle.float_decode(g, kind, imax, llr, early_stop=early, return_iters=True)
        assert res["1"][1] == ref_it
        np.testing.assert_array_equal(res["1"][0], ref)


def test_float_fold_absent_without_degree2(eng, reg_H):
    G = eng.Graph(graph.build_graph(reg_H), DEV)
    assert eng.FloatDecoder(G, 0, 5, 16, path="passes").folded == 0


# ------------------------------------------------------------------ channel-LLR precondition check
@pytest.mark.parametrize("path", ["auto", "passes"])
def test_float_input_check(eng, wlan_H, path):
    """ibl_float_input_check: the staging kernels count channel LLRs that break
    ibl_float_decode's precondition — BP fp64: NaN, |x| > ln(DBL_MAX) = 709.78 (where the reference's box-plus
    e^a overflows to NaN); BP fp32: NaN, +-inf (the value the decoder stages); min-sum: NaN only (+-inf is a
    known bit) — and the query returns IBL_EINVAL with the count; valid inputs count 0. The BP case with +-inf
    inputs is the one that failed in round 4 (gpurun_out/r4c2) before the precondition was narrowed."""
    from informationbottleneckdecodingldpc_amd._lib import IBLError
    g = graph.build_graph(wlan_H)
    G = eng.Graph(g, DEV)
    B = 96
    llr = _llrs(g, B, 1.5, seed=77)
    rng = np.random.default_rng(78)
    pos = rng.random(llr.shape) < 0.02
    bad_inf = llr.copy()
    bad_inf[pos] = np.where(rng.random(pos.sum()) < 0.8, np.inf, -np.inf)
    big = llr.copy()
    # fp64 BP: 709.8, -1e6, 1e30, 1e300 break |x| <= 709.78; fp32 BP: only 1e300 (inf once staged in fp32)
    big[0, :8] = [709.0, -709.0, 709.8, -1e6, 500.0, 1e30, 1e300, 709.78]
    nan = llr.copy()
    nan[3, 7] = np.nan
    for prec in (torch.float32, torch.float64):
        bp = eng.FloatDecoder(G, oracle.BP, 10, B, precision=prec, path=path)
        ms = eng.FloatDecoder(G, oracle.MINSUM, 10, B, precision=prec, path=path)
        for dec in (bp, ms):
            dec.decode(torch.from_numpy(llr).to(DEV).to(prec), early_stop=False)
            assert dec.input_violations() == 0
        bp.decode(torch.from_numpy(bad_inf).to(DEV).to(prec), early_stop=False)
        with pytest.raises(IBLError, match="BP precondition"):
            bp.input_violations()
        bp.decode(torch.from_numpy(bad_inf).to(DEV).to(prec), early_stop=False)
        assert bp.input_violations(raise_on_error=False) == int(pos.sum())
        assert bp.input_violations() == 0                       # cleared by the query
        ms.decode(torch.from_numpy(bad_inf).to(DEV).to(prec), early_stop=False)
        assert ms.input_violations() == 0                       # +-inf allowed for min-sum
        bp.decode(torch.from_numpy(big).to(DEV).to(torch.float64), early_stop=False)
        assert bp.input_violations(raise_on_error=False) == (4 if prec == torch.float64 else 1)
        bp.decode(torch.from_numpy(big.astype(np.float32)).to(DEV), early_stop=False)   # f32 caller values
        assert bp.input_violations(raise_on_error=False) == (4 if prec == torch.float64 else 1)
        for dec in (bp, ms):
            dec.decode(torch.from_numpy(nan).to(DEV).to(prec), early_stop=False)
            assert dec.input_violations(raise_on_error=False) == 1


def test_bp_large_finite_channel_llrs(eng, wlan_H):
    """BP takes every channel LLR the reference decodes without NaN. fp64: |x| up to ln(DBL_MAX) —
    e^(a+b) may overflow (the reference then gets log(inf) = inf, clamped to +-llr_max) while e^a does not — equals
    the fp64 oracle (1e-9) with no violation counted. fp32 (overflow-free box-plus): any finite value; channel
    values of +-1e30 decode like +-4000 (beyond any sum of clamped messages, so both clamp to +-llr_max in every
    message), so every APP LLR other than those channel positions' own equals the +-4000 decode, and theirs keep its
    sign."""
    g = graph.build_graph(wlan_H)
    G = eng.Graph(g, DEV)
    B = 64
    llr = _llrs(g, B, 1.5, seed=91)
    rng = np.random.default_rng(92)
    pos = rng.random(llr.shape) < 0.02
    sgn = np.where(rng.random(pos.sum()) < 0.8, 1.0, -1.0)
    big = llr.copy()
    big[pos] = sgn * rng.uniform(354.0, 709.78, pos.sum())
    big[0, :2] = [709.78, 709.78]                           # both inputs of one check near the limit
    dec = eng.FloatDecoder(G, oracle.BP, 15, B, precision=torch.float64)
    out = dec.decode(torch.from_numpy(big).to(DEV), early_stop=False)
    assert dec.input_violations() == 0
    ref = oracle.float_decode(g, oracle.BP, 15, big)
    o = out.cpu().numpy()
    assert not np.isnan(ref).any() and not np.isnan(o).any()
    np.testing.assert_allclose(o, ref, rtol=1e-15, atol=1e-9)
    f32 = eng.FloatDecoder(G, oracle.BP, 15, B, precision=torch.float32)
    huge, clip = llr.astype(np.float32), llr.astype(np.float32)
    huge[pos], clip[pos] = sgn * np.float32(1e30), sgn * np.float32(4000.0)
    oh = f32.decode(torch.from_numpy(huge).to(DEV), early_stop=False).cpu().numpy()
    assert f32.input_violations() == 0
    oc = f32.decode(torch.from_numpy(clip).to(DEV), early_stop=False).cpu().numpy()
    assert np.isfinite(oh).all()
    np.testing.assert_array_equal(oh[~pos], oc[~pos])
    assert ((oh[pos] < 0) == (oc[pos] < 0)).all()


def test_dropin_bp_raises_on_invalid_channel(wlan_H):
    """The reference-named BP class returning host arrays raises instead of handing back unspecified APP
    LLRs for +-inf channel values (kernels_min_and_BP.cl:5-9: the reference's box-plus gives NaN there)."""
    from informationbottleneckdecodingldpc_amd._lib import IBLError
    from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular
    g = graph.build_graph(wlan_H)
    llr = _llrs(g, 8, 1.5, 9)
    bp = BeliefPropagationDecoderClassIrregular(wlan_H, 20, 16, 8)
    bp.init_OpenCL_decoding(8)
    bp.decode_OpenCL_belief_propagation(llr)
    llr[5, 2] = np.inf
    with pytest.raises(IBLError):
        bp.decode_OpenCL_belief_propagation(llr)


# ------------------------------------------------------------------ small-batch per-pass kernels
@pytest.mark.parametrize("prec", [torch.float32, torch.float64])
@pytest.mark.parametrize("kind", [oracle.MINSUM, oracle.BP])
@pytest.mark.parametrize("name,imax,B,early,ebn0", [
    ("dvb", 12, 2, False, 1.0),        # the reference DVB-S2 driver's batch
    ("dvb", 30, 33, True, 2.0),        # ragged last word, early stop
    ("mixed", 6, 9, True, 2.0),        # every check degree 2..16, variable degree 1..16
    ("mixed", 6, 3, True, 2.0),        # every degree, tasks not contiguous, one word
    ("wlan", 10, 1, False, 1.5),       # B = 1
    ("wlan", 20, 70, True, 1.5)])      # forced onto the small kernels past the default threshold
def test_float_small_batch_kernels(eng, prec, kind, name, imax, B, early, ebn0, wlan_H, dvb_H):
    """The small-batch float kernels (fl_*_small: wave item = up to 64 same-degree nodes x one 16-byte word) give
    the per-pass kernels' bits and stop iteration (small_b = 0 runs those, with the fold where it applies); fp64
    min-sum also equals the oracle."""
    H = {"dvb": dvb_H, "wlan": wlan_H}.get(name)
    if H is None:
        H = mixed_code(np.arange(2, 17), np.arange(1, 17), 600, seed=15)
    g = graph.build_graph(H)
    G = eng.Graph(g, DEV)
    llr = _llrs(g, B, ebn0, seed=imax + 13 * B, quantised=True)
    res = {}
    for small_b in (1024, 0):
        dec = eng.FloatDecoder(G, kind, imax, B, precision=prec, path="passes")
        dec.small_batch = small_b
        it = torch.zeros(1, dtype=torch.int32, device=DEV)
        out = dec.decode(torch.from_numpy(llr).to(DEV).to(prec), early_stop=early, iters=it)
        res[small_b] = (out.double().cpu().numpy(), int(it.item()))
    assert res[1024][1] == res[0][1]
    np.testing.assert_array_equal(res[1024][0], res[0][0])
    if kind == oracle.MINSUM and prec == torch.float64:
        ref, ref_it = oracle.float_decode(g, kind, imax, llr, early_stop=early, return_iters=True)
        assert res[1024][1] == ref_it
        np.testing.assert_array_equal(res[1024][0], ref)


def test_float_small_batch_default(eng, dvb_H):
    G = eng.Graph(graph.build_graph(dvb_H), DEV)
    assert eng.FloatDecoder(G, 1, 5, 16).small_batch == 64
