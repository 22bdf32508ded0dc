"""The kernel path each bench line times, checked against the oracle directly.

The small-batch float kernels (round 5) take every batch B <= 64, so the DVB-S2 float tests of
test_gpu_float.py (B = 4..16) run those kernels, not the folded per-pass kernels that BASELINE C5 times
at B = 8192. These tests build each config's decoder through bench.py's own `build_decoder` (same
arguments, same tables, same channel stream) and

  * assert which path decodes (fused / small-batch / per-pass, degree-2 variables folded) for C1-C5;
  * compare C5's path (DVB-S2 BP fp32, i_max = 100, folded per-pass kernels) with the fp64 oracle of
    kernels_min_and_BP.cl:5-123 (|x-y| <= 1e-5 max(|x|,|y|) + 1e-4, no hard flips, same stop
    iteration): spread columns of the bench's own 8192-codeword batch with fixed iterations, and whole
    batches of 96 with early stop (one that never stops, one that stops before i_max - 1);
  * compare fp32 min-sum on the same folded per-pass path with the fp32 oracle bit for bit.

Codewords are independent under fixed iterations, so columns of the full batch can be checked alone; with
early stop the stop is batch-global, so those batches are checked whole.
"""
import numpy as np
import pytest
import torch

import bench
from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
REL, TOL_ABS = 1e-5, 1e-4


@pytest.fixture(scope="module")
def eng():
    from informationbottleneckdecodingldpc_amd import engine
    return engine


@pytest.fixture(scope="module")
def dvb_setup(eng):
    """bench.py's DVB-S2 setup payload, host graph and device graph (shared by the DVB-S2 cases)."""
    a = bench.parse(["--config", "C5"])
    arrays = bench.setup_arrays(a)
    g = bench.graph_of(arrays)
    return arrays, g, eng.Graph(g, DEV)


def _h5(out, ref):
    return np.abs(out - ref) > REL * np.maximum(np.abs(out), np.abs(ref)) + TOL_ABS


def _hard_flips(out, ref):
    return int((((out < 0) != (ref < 0)) & (np.abs(ref) > REL * np.abs(ref) + TOL_ABS)).sum())


def _bench_decoder(eng, argv, setup=None):
    a = bench.parse(argv)
    if setup is None:
        arrays = bench.setup_arrays(a)
        g = bench.graph_of(arrays)
        G = eng.Graph(g, DEV)
    else:
        arrays, g, G = setup
    q = UniformQuantizer(sigma2_from_ebn0(a.ebn0, g.R_c), 16)
    B = a.batch_per_gpu
    dec, match = bench.build_decoder(a, G, g, arrays, q, B)
    return a, g, q, B, dec, bench.decoder_path(a, dec, B)


def _bench_llrs(eng, g, q, B):
    """The bench's float channel: device Philox key CH_SEED at global batch 0, cluster LLRs in fp32."""
    llr = torch.empty((g.n_v, B), dtype=torch.float32, device=DEV)
    eng.channel_sample(llr, q.cdf_t_given_x_equals_zero, bench.CH_SEED, 0, llr=q.output_LLRs)
    return llr


def _decode(dec, x, early):
    it = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = dec.decode(x, early_stop=early, iters=it)
    torch.cuda.synchronize()
    return out, int(it.item())


def _spread(B, n):
    return np.unique(np.concatenate([np.linspace(0, B - 1, n).astype(np.int64), [B - 1]]))


@pytest.mark.parametrize("config,expect", [
    ("C1", "fused on-chip kernel"), ("C2", "fused on-chip kernel"), ("C3", "fused on-chip kernel"),
    ("C4", "per-pass kernels"), ("C5", "per-pass kernels")])
@pytest.mark.parametrize("early", [False, True])
def test_bench_configs_run_their_kernel_paths(eng, dvb_setup, config, expect, early):
    """Every BASELINE config's bench decoder decodes its batch on the path the bench line names: C1/C2 on
    the fused on-chip IB kernel, C3 on the fused min-sum kernel, C4 on the IB per-pass fast kernels (not the
    small-batch ones), C5 on the per-pass float kernels with all 32,399 degree-2 variables folded."""
    argv = ["--config", config] + (["--early-stop"] if early else [])
    a, g, q, B, dec, p = _bench_decoder(eng, argv, dvb_setup if config == "C5" else None)
    assert p["name"] == expect, (config, p)
    if config == "C4":
        assert dec.fast_path and not p["small"] and B > dec.small_batch
    if config == "C5":
        assert not p["small"] and B > dec.small_batch
        assert p["folded"] == dec.folded == 32399
    del dec


def test_c5_bench_path_bp_fp32_columns_vs_oracle(eng, dvb_setup):
    """BASELINE C5 exactly as bench.py times it (DVB-S2 BP fp32, i_max = 100, B = 8192, fixed iterations, the
    folded per-pass kernels): 48 spread columns of the bench's own batch against the fp64 oracle within H5."""
    a, g, q, B, dec, p = _bench_decoder(eng, ["--config", "C5"], dvb_setup)
    assert B == 8192 and p["name"] == "per-pass kernels" and p["folded"] == 32399
    llr = _bench_llrs(eng, g, q, B)
    out, it = _decode(dec, llr, False)
    assert it == 99
    cols = _spread(B, 48)
    x = llr[:, cols].cpu().numpy().astype(np.float64)
    ref = oracle.float_decode(g, oracle.BP, 100, x)
    o = out[:, cols].cpu().numpy().astype(np.float64)
    bad = _h5(o, ref)
    print(f"C5 bench path: {len(cols)} columns, max |x-y| {np.abs(o - ref).max():.3e}, decided errors "
          f"{int((ref[:g.data_len] < 0).sum())}")
    assert bad.sum() == 0, f"{bad.sum()} of {bad.size} LLRs outside H5, max |x-y| {np.abs(o - ref).max():.3e}"
    assert _hard_flips(o, ref) == 0


def _force_degree1_reliable(g, q, llr):
    """The batch-global syndrome (on the variable-to-check messages, kernels_min_and_BP.cl:206-227) includes the
    checks around DVB-S2's degree-1 parity variable, whose message is its channel value: with a weak or wrong one
    the staircase neighbour's extrinsic message to its other check can keep the wrong sign forever although every
    decision is right (measured with the oracle: one unsatisfied check from iteration 18 on at 3 dB). Giving that
    variable the most reliable positive cluster LLR lets a decodable batch stop."""
    d1 = np.nonzero(np.asarray(g.vn_deg) == 1)[0]
    assert d1.size >= 1
    llr[torch.from_numpy(d1).to(llr.device)] = float(np.max(q.output_LLRs))
    return llr


@pytest.mark.parametrize("ebn0,stops", [(1.0, False), (3.0, True)])
def test_c5_bench_path_bp_fp32_early_stop_vs_oracle(eng, dvb_setup, ebn0, stops):
    """C5's decoder state with early stop (`bench.py --config C5 --early-stop`; fold mode 2: folded outputs also
    reach the variable inbox, since any pass may be the last) on whole batches of 96 > small_batch: APP LLRs
    within H5 of the fp64 oracle, no hard flips, the same stop iteration — at 1.0 dB (the batch never stops)
    and at 3.0 dB with the degree-1 variable's channel value made reliable (the batch stops early)."""
    a, g, q, B, dec, p = _bench_decoder(eng, ["--config", "C5", "--early-stop", "--batch-per-gpu", "96",
                                              "--ebn0", str(ebn0)], dvb_setup)
    assert B == 96 > dec.small_batch and p["name"] == "per-pass kernels" and p["folded"] == 32399
    llr = _bench_llrs(eng, g, q, B)
    if stops:
        llr = _force_degree1_reliable(g, q, llr)
    out, it = _decode(dec, llr, True)
    x = llr.cpu().numpy().astype(np.float64)
    ref, ref_it = oracle.float_decode(g, oracle.BP, 100, x, early_stop=True, return_iters=True)
    assert it == ref_it
    assert (ref_it < 99) == stops, ref_it
    o = out.cpu().numpy().astype(np.float64)
    bad = _h5(o, ref)
    assert bad.sum() == 0, f"{bad.sum()} of {bad.size} LLRs outside H5, max |x-y| {np.abs(o - ref).max():.3e}"
    assert _hard_flips(o, ref) == 0


def test_minsum_fp32_dvbs2_folded_path_columns_bit_exact(eng, dvb_setup):
    """fp32 min-sum on the DVB-S2 code through the folded per-pass kernels (B = 8192, i_max = 50, fixed
    iterations): 64 spread columns bit-identical to the fp32 oracle (kernels_min_and_BP.cl:76-167 in IEEE
    single, the same selections and ordered adds)."""
    a, g, q, B, dec, p = _bench_decoder(eng, ["--code", "dvbs2", "--kind", "minsum", "--imax", "50"], dvb_setup)
    assert B == 8192 and p["name"] == "per-pass kernels" and p["folded"] == 32399
    llr = _bench_llrs(eng, g, q, B)
    out, it = _decode(dec, llr, False)
    assert it == 49
    cols = _spread(B, 64)
    ref = oracle.float32_decode(g, 50, llr[:, cols].cpu().numpy())
    np.testing.assert_array_equal(out[:, cols].cpu().numpy(), ref)


@pytest.mark.parametrize("ebn0,stops", [(1.0, False), (3.0, True)])
def test_minsum_fp32_dvbs2_folded_path_early_stop_bit_exact(eng, dvb_setup, ebn0, stops):
    """The same folded per-pass min-sum path with early stop on whole batches of 100: bit-identical APP LLRs
    and stop iteration against the fp32 oracle."""
    a, g, q, B, dec, p = _bench_decoder(eng, ["--code", "dvbs2", "--kind", "minsum", "--imax", "50",
                                              "--batch-per-gpu", "100", "--early-stop", "--ebn0", str(ebn0)],
                                        dvb_setup)
    assert B == 100 > dec.small_batch and p["name"] == "per-pass kernels" and p["folded"] == 32399
    llr = _bench_llrs(eng, g, q, B)
    if stops:
        llr = _force_degree1_reliable(g, q, llr)
    out, it = _decode(dec, llr, True)
    ref, ref_it = oracle.float32_decode(g, 50, llr.cpu().numpy(), early_stop=True, return_iters=True)
    assert it == ref_it
    assert (ref_it < 49) == stops, ref_it
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
