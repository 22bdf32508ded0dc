"""CPU: the discrete-density-evolution table generator (tables.de_tables, round 6).

The reference designs its decoders by discrete density evolution with an information-bottleneck quantiser per
partial node operation and iteration, and information matching between the node degrees
(Discrete_LDPC_decoding/Discrete_Density_Evolution_irreg.py:75-432, Information_Matching.py:29-71); its ib_base
package is absent, so parity with the published tables is unpinned. These tests pin what the generator must hold:
the reference layout, the symmetry every symmetric decoder's tables have, a DE trajectory that converges above
the threshold and stalls below it, and — decoded by the oracle (a restatement of kernels_template_irreg.cl) — a
decoder that beats the fixed-alphabet LLR tables on the same frames.
"""
import numpy as np
import pytest

from informationbottleneckdecodingldpc_amd import codes, graph, tables
from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0
from oracle import oracle


@pytest.fixture(scope="module")
def wlan1944():
    return graph.build_graph(codes.wlan_80211n(81))


def _design(g, ebn0, imax, **kw):
    q = UniformQuantizer(sigma2_from_ebn0(ebn0, g.R_c), 16)
    rho, lam = tables.edge_degree_distributions(g)
    return tables.de_tables(q.p_t_given_x0, q.output_LLRs, rho, lam, imax, **kw), q


def test_edge_degree_distributions(wlan1944):
    rho, lam = tables.edge_degree_distributions(wlan1944)
    assert sorted(rho) == [7, 8] and sorted(lam) == [2, 3, 4, 11]
    assert abs(sum(rho.values()) - 1) < 1e-12 and abs(sum(lam.values()) - 1) < 1e-12
    assert rho[7] == pytest.approx(7 * np.sum(wlan1944.cn_deg == 7) / wlan1944.n_e)


def test_de_tables_layout_and_symmetry(wlan1944):
    """Reference lengths and ranges (IBTables.check), and the symmetry of a symmetric decoder: a check op's output
    mirrors (t -> T-1-t) when either input mirrors, a variable op's when both do, and every matching vector maps
    mirrored clusters to mirrored clusters."""
    g = wlan1944
    imax, T, CM, VM = 12, 16, g.d_c_max, g.d_v_max
    (tb, tr), _ = _design(g, 2.0, imax, return_trace=True)
    tb.check()
    assert tb.cn.size == tables.cn_lut_len(T, T, CM, imax) and tb.vn.size == tables.vn_lut_len(T, T, VM, imax)
    cn0 = tb.cn[:T * T].reshape(T, T)
    assert np.array_equal(cn0[::-1], T - 1 - cn0) and np.array_equal(cn0, cn0.T)
    off = T * T + (CM - 3) * T * T
    for k in range(imax - 1):
        for l in range(CM - 2):
            o = off + k * (CM - 2) * T * T + l * T * T
            blk = tb.cn[o:o + T * T].reshape(T, T)
            assert np.array_equal(blk[::-1], T - 1 - blk) and np.array_equal(blk[:, ::-1], T - 1 - blk)
    for k in range(imax):
        o = k * (T * T + (VM - 1) * T * T)
        for l in range(VM):
            blk = tb.vn[o + l * T * T:o + (l + 1) * T * T].reshape(T, T)
            assert np.array_equal(blk[::-1, ::-1], T - 1 - blk)
    mc = tb.match_cn.reshape(imax, CM, T)
    mv = tb.match_vn.reshape(imax, VM, T)
    for m in list(mc.reshape(-1, T)) + list(mv.reshape(-1, T)):
        assert np.array_equal(m[::-1], T - 1 - m) and np.all(np.diff(m) >= 0)    # monotone: order kept
    # every matched alphabet is a valid symmetric one: mutual information grows over the iterations at 2 dB
    assert np.all(np.diff(tr["I_vn"]) > -1e-9) and tr["I_vn"][-1] > 0.98


def test_de_trajectory_threshold():
    """DE on the DVB-S2 profile (the build's structured N=64800 code): at 1.2 dB the variable-output mutual
    information reaches > 0.99 within 50 iterations, at 0.5 dB it stalls below 0.65 (a fixed point)."""
    g = graph.build_graph(codes.dvbs2_structured(seed=0))
    (_, hi), _ = _design(g, 1.2, 50, return_trace=True)
    (_, lo), _ = _design(g, 0.5, 50, return_trace=True)
    assert hi["I_vn"][-1] > 0.99
    assert lo["I_vn"][-1] < 0.65 and abs(lo["I_vn"][-1] - lo["I_vn"][-10]) < 5e-3


def test_de_tables_decode_better_than_fixed_alphabet(wlan1944):
    """The oracle decoder (kernels_template_irreg.cl restated) with DE tables designed at 1.5 dB against the round-5
    fixed-alphabet LLR tables, same frames (WLAN N=1944, i_max=20, 256 codewords): fewer bit errors at 1.5 dB, and
    no errors at 2.5 dB."""
    g = wlan1944
    de, q = _design(g, 1.5, 20)
    llr = tables.llr_tables(q.output_LLRs, g.d_c_max, g.d_v_max, 20)
    errs = {}
    for ebn0 in (1.5, 2.5):
        qq = UniformQuantizer(sigma2_from_ebn0(ebn0, g.R_c), 16)
        ch = oracle.channel_sample(qq.cdf_t_given_x_equals_zero, 3, 0, g.n_v, 256)
        for name, tb in (("de", de), ("llr", llr)):
            out = oracle.ib_decode(g, tb, ch, match=True)
            errs[(ebn0, name)] = int((out[:g.data_len] < 8).sum())
    assert errs[(1.5, "de")] < 0.8 * errs[(1.5, "llr")], errs
    assert errs[(2.5, "de")] == 0, errs


def test_de_tables_regular_code_without_matching():
    """A regular code has one degree per side, so the decoder needs no matching (the reference's regular class has
    none): the DE tables decode the (3,6) N=8000 code (BASELINE C1/C2) at 2.0 dB without errors on 16 codewords."""
    g = graph.build_graph(codes.regular_code(8000, 3, 6, seed=0))
    tb, q = _design(g, 1.5, 30, match=False)
    assert np.array_equal(tb.match_cn, tables.identity_matching(16, g.d_c_max, 30))
    qq = UniformQuantizer(sigma2_from_ebn0(2.0, g.R_c), 16)
    ch = oracle.channel_sample(qq.cdf_t_given_x_equals_zero, 4, 0, g.n_v, 16)
    out = oracle.ib_decode(g, tb, ch, match=False)
    assert int((out < 8).sum()) == 0
