"""GPU parity of the float min-sum / BP decoders against the fp64 CPU oracle (a restatement of
kernels_min_and_BP.cl; the reference's own float host path is broken, SURVEY Appendix C3, so
parity is pinned by the kernel text).

Bars (written in the tests):
  * fp64 min-sum: bit-identical APP LLRs and stop iteration;
  * fp64 BP: |x-y| <= 1e-9 (device exp/log vs glibc differ in the last ulps);
  * fp32 vs the fp64 oracle (BASELINE: "within 1e-5 relative"): |x-y| <= 1e-5*max(|x|,|y|) +
    TOL_ABS for >= 99.9 % of APP LLRs and identical hard decisions wherever |oracle LLR| >
    HARD_EPS — for BP at every i_max tested, for min-sum up to i_max = 10. Unnormalised min-sum
    on the reference's 16-level quantised LLR alphabet is chaotic past ~20 iterations: sums that
    cancel exactly to 0 in fp64 (sign() = 0 kills a message) come out as +-1 ulp in fp32, and the
    trajectories separate (measured: tools/diag_float32.py). There the bar is the decoder's
    output statistic — the bit-error count — within sampling noise (test_float32_minsum_ber).
"""
import numpy as np
import pytest
import torch

from informationbottleneckdecodingldpc_amd import graph
from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
REL = 1e-5
TOL_ABS = {0: 1e-4, 1: 2e-3}      # min-sum: fp32 sums of LLRs; BP: + fp32 log/exp per box-plus
HARD_EPS = 1e-2


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


@pytest.mark.parametrize("kind,name,imax,B,ebn0", [
    (oracle.MINSUM, "wlan", 10, 256, 1.5), (oracle.MINSUM, "reg", 10, 70, 2.0), (oracle.MINSUM, "dvb", 10, 8, 1.2),
    (oracle.BP, "wlan", 10, 256, 1.5), (oracle.BP, "wlan", 50, 100, 2.0), (oracle.BP, "reg", 20, 70, 2.0),
    (oracle.BP, "dvb", 10, 8, 1.2)])
def test_float32_vs_oracle(eng, kind, name, imax, B, ebn0, wlan_H, reg_H, dvb_H):
    g = graph.build_graph({"wlan": wlan_H, "reg": reg_H, "dvb": dvb_H}[name])
    llr = _llrs(g, B, ebn0, seed=3 * imax + B, quantised=True)
    ref = oracle.float_decode(g, kind, imax, llr)
    out, _ = _gpu(eng, g, kind, imax, llr, torch.float32, False)
    tol = REL * np.maximum(np.abs(out), np.abs(ref)) + TOL_ABS[kind]
    bad = np.abs(out - ref) > tol
    assert bad.mean() < 1e-3, f"{bad.sum()} of {bad.size} LLRs outside tolerance"
    hard_diff = ((out < 0) != (ref < 0)) & (np.abs(ref) > HARD_EPS)
    assert hard_diff.sum() == 0


def test_float32_minsum_ber(eng, wlan_H):
    """i_max = 50 fp32 min-sum: bit-error count vs the fp64 oracle within sampling noise."""
    g = graph.build_graph(wlan_H)
    llr = _llrs(g, 400, 2.0, seed=77)
    ref = oracle.float_decode(g, oracle.MINSUM, 50, llr)
    out, _ = _gpu(eng, g, oracle.MINSUM, 50, llr, torch.float32, False)
    e_ref = int((ref[:g.data_len] < 0).sum())
    e_gpu = int((out[:g.data_len] < 0).sum())
    assert abs(e_gpu - e_ref) <= max(10, 4 * np.sqrt(e_ref + 1)), (e_gpu, e_ref)


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
