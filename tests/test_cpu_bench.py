"""CPU: bench.py's measurement arithmetic (no GPU): SURVEY §8(d) bytes per codeword and the roofline
objects — priced at the bytes each kernel moves, so frac = achieved / peak <= 1 for physical timings."""
import types

import numpy as np
import pytest

import bench
from informationbottleneckdecodingldpc_amd import codes, graph


def _args(**kw):
    a = types.SimpleNamespace(kind="ib", pmc="/nonexistent", config=None)
    a.__dict__.update(kw)
    return a


def test_bytes_per_codeword_dvbs2():
    # i_max (4E + N) + 2N with u8 messages: 48.73 MB at i_max = 50
    assert bench.bytes_per_cw(226799, 64800, 50, 1) == 50 * (4 * 226799 + 64800) + 2 * 64800
    assert abs(bench.bytes_per_cw(226799, 64800, 50, 1) / 1e6 - 48.73) < 0.01


@pytest.fixture(scope="module")
def dvb():
    return graph.build_graph(codes.dvbs2_structured(seed=0))


def test_ib_fast_roofline_prices_u4_bytes(dvb):
    g, B = dvb, 8192
    r = bench.roofline(_args(), g, g.n_v, B, 50, 1, 0.5, "u4", True, False,
                       cn_avg=0.464, vn_avg=0.458, cn_ms=0.464 * 50, vn_ms=0.458 * 49, cn_n=50, vn_n=49, dec=None)
    assert r["bound"] == "hbm" and r["format"] == "u4"
    # the CN pass (50 launches) dominates: E*B/2 read + E*B/2 written
    assert r["kernel"] == "ib_cn_fast" and r["bytes_per_launch"] == g.n_e * B
    assert r["frac"] == pytest.approx(g.n_e * B / 0.464e-3 / 1e9 / bench.HBM_PEAK_GBPS, rel=1e-3)
    assert 0 < r["frac"] <= 1
    assert r["u8_equivalent"]["bytes_per_launch"] == 2 * g.n_e * B
    lk = r["lds_lookups_per_clk_per_cu"]
    assert lk["ceiling"] == 32.0 and 0 < lk["cn"] < 32 and 0 < lk["vn"] < 32


def test_fused_rooflines_are_lds_bound():
    g = graph.build_graph(codes.regular_code(8000, 3, 6, seed=0))
    r = bench.roofline(_args(), g, g.n_v, 65536, 50, 1, 0.5, "u4", False, True,
                       cn_avg=37.5, vn_avg=0.0, cn_ms=37.5, vn_ms=0.0, cn_n=1, vn_n=0, dec=None)
    assert r["bound"] == "lds" and r["kernel"] == "ib_fused" and 0 < r["frac"] <= 1
    w = graph.build_graph(codes.wlan_80211n(81))
    f = bench.roofline(_args(kind="minsum"), w, w.n_v, 262144, 50, 4, 4, "f32", False, True,
                       cn_avg=55.3, vn_avg=0.0, cn_ms=55.3, vn_ms=0.0, cn_n=1, vn_n=0, dec=None)
    assert f["bound"] == "lds" and f["kernel"] == "fl_fused" and 0 < f["frac"] <= 1
    # LDS peak at the 16-byte slot mix lies between the write (79 B/clk) and read (256 B/clk) rates
    per_clk = f["peak"] / (bench.NUM_CUS * bench.LDS_CLK_GHZ)
    assert 79 <= per_clk <= 256


def test_numpy_host_baseline_workers(tmp_path):
    """The spawned numpy decode_on_host workers reproduce the in-process decoder."""
    from informationbottleneckdecodingldpc_amd import tables
    from oracle.host_numpy import HostDecoder
    g = graph.build_graph(codes.regular_code(504, 3, 6, seed=7))
    tb = tables.random_tables(16, 16, 6, 3, 4, seed=2)
    x = np.random.default_rng(0).integers(0, 16, (g.n_v, 6)).astype(np.int32)
    outs, per_core, agg, wall, per_core_f = bench.numpy_host_baseline(g, tb, x, 4, True, 2)
    ref = HostDecoder(g, 16, 16, 4, tb.cn, tb.vn, regular=True)
    for k in range(6):
        np.testing.assert_array_equal(outs[:, k], ref.decode(x[:, k]))
    assert per_core > 0 and agg > 0 and wall > 0 and per_core_f > 0


def test_committed_pmc_traffic_feeds_the_headline(dvb):
    """profiles/pmc_traffic.json (bench.py's default --pmc) is in the schema bench.py reads, so the
    headline line carries the measured per-launch HBM bytes of its dominant kernel (roofline.traffic),
    and they lie within 2 % of the stored algorithmic bytes (no wasted re-reads)."""
    import os
    g, B = dvb, 8192
    pmc = os.path.join(os.path.dirname(bench.__file__), "profiles", "pmc_traffic.json")
    r = bench.roofline(_args(pmc=pmc), g, g.n_v, B, 50, 1, 0.5, "u4", True, False,
                       cn_avg=0.464, vn_avg=0.458, cn_ms=0.464 * 50, vn_ms=0.458 * 49, cn_n=50, vn_n=49, dec=None)
    assert r["traffic"] is not None
    assert abs(r["traffic"] / r["bytes_per_launch"] - 1) < 0.02


def test_moved_bytes_dvbs2_u4(dvb):
    """The headline's hbm_gbps_algorithmic prices the bytes the per-pass u4 path moves per codeword:
    stage N (u8 in) + N/2, check pass 0 2E/2, 49 x (4E + N)/2, decision (E + N)/2 + N (u8 out)."""
    g = dvb
    E, N = g.n_e, g.n_v
    m = bench.moved_bytes_per_cw(E, N, 50, "passes", 0.5, 1, 1)
    assert m == N + N / 2 + E + 49 * (4 * E + N) / 2 + (E + N) / 2 + N
    assert abs(m / 1e6 - 24.35) < 0.01
    # at the round-2 headline rate this is physically possible, while the u8 figure was not
    assert 175e3 * m / 1e9 < bench.HBM_PEAK_GBPS < 175e3 * bench.bytes_per_cw(E, N, 50, 1) / 1e9
    # float per-pass: send reads N and writes E instead of the gather; 99 check passes, 98 variable passes
    # (the last iteration's variable pass feeds nothing and is not run)
    f = bench.moved_bytes_per_cw(E, N, 100, "passes", 4, 4, 4)
    assert f == 4 * N + 4 * N + 4 * (E + N) + 4 * (99 * 2 * E + 98 * (2 * E + N)) + 4 * (E + N) + 4 * N
    # with the degree-2 fold (C5: 32,399 variables): 98 folding check passes read 2 channel rows per folded
    # variable; the 98 variable passes cover E - 2 nf edges and N - nf variables
    nf = 32399
    ff = bench.moved_bytes_per_cw(E, N, 100, "passes", 4, 4, 4, folded=nf)
    assert ff == f + 4 * 98 * (2 * nf - 4 * nf - nf)
    assert 0.88 < ff / f < 0.92                       # ~10 % fewer bytes per codeword
    # fused: channel in, staging copy written and read, output out
    assert bench.moved_bytes_per_cw(E, N, 50, "fused", 0.5, 1, 1, w_stage=1) == 4 * N


def test_float_roofline_with_fold(dvb):
    """The per-pass float roofline prices both passes; with the fold the variable pass moves E - 2 nf edge
    rows (read + write) and N - nf channel rows, and the folding check passes read 2 nf channel rows."""
    g, B, nf = dvb, 8192, 32399
    r = bench.roofline(_args(kind="bp"), g, g.n_v, B, 100, 4, 4, "f32", False, False,
                       cn_avg=3.2, vn_avg=2.2, cn_ms=3.2 * 99, vn_ms=2.2 * 98, cn_n=99, vn_n=98, dec=None, folded=nf)
    assert r["passes"]["vn"]["bytes_per_launch"] == (2 * (g.n_e - 2 * nf) + g.n_v - nf) * 4 * B
    assert r["passes"]["cn"]["bytes_per_launch"] == round((2 * g.n_e + 2 * nf * 98 / 99) * 4 * B)
    assert r["kernel"] == "fl_cn" and r["folded_degree2_variables"] == nf
    assert 0 < r["passes"]["cn"]["frac"] <= 1 and 0 < r["passes"]["vn"]["frac"] <= 1


def test_committed_bench_lines_are_physical():
    """Every bench line committed from round 3 on reports top-level HBM GB/s at or below the HBM peak
    (rounds 1-2 priced that field at the u8-equivalent width; it is now hbm_gbps_u8_equivalent)."""
    import glob
    import json
    import os
    import re
    prof = os.path.join(os.path.dirname(bench.__file__), "profiles")
    seen = 0
    for p in sorted(glob.glob(os.path.join(prof, "r*_bench*.json"))):
        m = re.match(r"r(\d+)_", os.path.basename(p))
        if not m or int(m.group(1)) < 3:
            continue
        with open(p) as fh:
            for ln in fh:
                ln = ln.strip()
                if not ln.startswith("{"):
                    continue
                d = json.loads(ln)
                assert d["hbm_gbps_algorithmic"] <= bench.HBM_PEAK_GBPS, p
                assert d["roofline"]["frac"] <= 1.0, p
                seen += 1
    assert seen >= 5          # at least the five round-3 config lines (C1-C5)


def test_measured_lookup_ceiling_from_profile():
    """bench.py reports the LDS lookup-chain rate the committed microbenchmark measured beside the nominal
    32/clk/CU ceiling (LDS-only rows of profiles/r03_ubench_lookup_rate.json)."""
    import bench
    mc = bench.measured_lookup_ceiling()
    assert mc is not None and 20.0 < mc <= 32.0


def test_bench_arguments(monkeypatch):
    """Presets keep an explicit --batch-per-gpu; --early-stop moves the default Eb/N0 to SURVEY §8(d)'s 1.0 dB."""
    import sys
    monkeypatch.setattr(sys, "argv", ["bench.py", "--config", "C4", "--early-stop", "--batch-per-gpu", "32"])
    a = bench.parse()
    assert (a.code, a.kind, a.imax, a.batch_per_gpu, a.ebn0, a.early_stop) == ("dvbs2", "ib", 50, 32, 1.0, True)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--config", "C5"])
    a = bench.parse()
    assert (a.kind, a.imax, a.batch_per_gpu, a.ebn0, a.early_stop, a.sub_batch, a.batch_offset) == \
        ("bp", 100, 8192, 0.6, False, 0, 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--config", "C1", "--ebn0", "2.5"])
    a = bench.parse()
    assert a.no_match and a.ebn0 == 2.5 and a.batch_per_gpu == 1000
