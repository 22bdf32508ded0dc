"""CPU: host-side components — loaders, generators, tables, channel model, the C ABI's exported
symbols and host-only index construction, the drop-in classes' set-up, and the fail-loudly rule."""
import os
import re
import sys

import numpy as np
import pytest
import scipy.sparse as sp

from informationbottleneckdecodingldpc_amd import codes, graph, tables
from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from informationbottleneckdecodingldpc_amd import _build, _lib
    if not os.path.exists(_lib.LIB_PATH):
        _build.build()
    return _lib


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "ibldpc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ibl_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_header_symbol(lib):
    L = lib.load()
    syms = header_symbols()
    assert len(syms) >= 19
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(lib.EXPORTS) == syms
    assert L.ibl_version() == 3


def test_product_library_has_no_diagnostic_hooks(lib):
    """The timing-only hooks (IBL_VN_PART runs part of the variable pass: its outputs are not decodes;
    IBL_TRACE_WAVES / IBL_TRACE_FUSED allocate and sync per decode; IBL_DEBUG_SYNC syncs per launch) exist
    only in diagnostic builds (-DIBL_DIAG=1, tools/variants.py diag / ftrace): the product library does not
    even hold their names, so no environment variable can change what a decode computes or costs. The
    create-time A/B knobs stay (read once per decoder)."""
    from informationbottleneckdecodingldpc_amd import _build
    _build.build()
    blob = open(lib.LIB_PATH, "rb").read()
    for name in (b"IBL_VN_PART", b"IBL_TRACE_WAVES", b"IBL_TRACE_FUSED", b"IBL_DEBUG_SYNC"):
        assert name not in blob, name
    src = open(os.path.join(ROOT, "informationbottleneckdecodingldpc_amd", "csrc", "capi.hip")).read()
    # every getenv outside the diagnostic blocks sits in a create-time function
    body = re.sub(r"#if IBL_DIAG.*?#endif", "", src, flags=re.S)
    decode_fns = re.findall(r"\nint (ibl_(?:ib|float)_decode)\(.*?\n}\n", body, flags=re.S)
    assert len(decode_fns) == 2
    for m in re.finditer(r"\nint (ibl_(?:ib|float)_decode)\(.*?\n}\n", body, flags=re.S):
        assert "getenv" not in m.group(0), m.group(1)
    ncw = re.search(r"int ib_fused_ncw\(.*?\n}\n", body, flags=re.S).group(0)
    assert "getenv" not in ncw


def test_library_device_count_without_gpu(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    assert lib.device_count() == 0


@pytest.mark.parametrize("name", ["reg", "wlan"])
def test_capi_map_node_connections_equals_reference(lib, golden, reg_H, wlan_H, name):
    """Host-only C ABI entry (no device call) reproduces the reference's index arrays."""
    H = reg_H if name == "reg" else wlan_H
    A = codes.canonical_csr(H)
    out = lib.map_node_connections(A.shape[1], A.shape[0], A.indptr, A.indices)
    for k, v in out.items():
        np.testing.assert_array_equal(v, golden[f"{name}_idx_{k}"], err_msg=k)


def test_capi_rejects_non_canonical_csr(lib):
    with pytest.raises(lib.IBLError):
        lib.map_node_connections(3, 1, np.array([0, 2]), np.array([2, 1]))
    with pytest.raises(lib.IBLError):
        lib.map_node_connections(3, 1, np.array([0, 2]), np.array([0, 5]))


def test_capi_dvbs2_matches_python_graph(lib, dvb_H):
    g = graph.build_graph(dvb_H)
    out = lib.map_node_connections(g.n_v, g.n_c, g.csr_indptr, g.csr_cols)
    for k, v in out.items():
        np.testing.assert_array_equal(v, getattr(g, k), err_msg=k)


def test_loaders_round_trip(tmp_path, reg_H):
    A = codes.canonical_csr(reg_H)
    np.save(tmp_path / "h.npy", A.toarray())
    codes.save_sparse_csr(str(tmp_path / "h.npz"), A)
    # alist with weight lines
    M, N = A.shape
    csc = A.tocsc()
    vdeg, cdeg = np.diff(csc.indptr), np.diff(A.indptr)
    lines = [f"{N} {M}", f"{vdeg.max()} {cdeg.max()}", " ".join(map(str, vdeg)), " ".join(map(str, cdeg))]
    for j in range(N):
        r = csc.indices[csc.indptr[j]:csc.indptr[j + 1]] + 1
        lines.append(" ".join(map(str, np.pad(r, (0, vdeg.max() - r.size)))))
    (tmp_path / "h.alist").write_text("\n".join(lines) + "\n")
    for f in ("h.npy", "h.npz", "h.alist"):
        B = codes.load_check_mat(str(tmp_path / f))
        assert (B != A).nnz == 0, f


def test_regular_code_is_simple_and_regular():
    H = codes.regular_code(8000, 3, 6, seed=0)
    g = graph.build_graph(H)
    assert (g.n_c, g.n_v, g.n_e) == (4000, 8000, 24000)
    assert set(g.cn_deg) == {6} and set(g.vn_deg) == {3}
    assert g.R_c == 0.5 and g.data_len == 4000


def test_wlan_z81_structure():
    g = graph.build_graph(codes.wlan_80211n(81))
    assert (g.n_c, g.n_v) == (972, 1944)
    assert set(g.cn_deg) == {7, 8} and set(g.vn_deg) == {2, 3, 4, 11}
    # the standard's Z=81 table (not held by the reference): same column weights as the Z=54
    # table, the dual-diagonal parity part, and girth >= 6 after lifting (no 4-cycles)
    b81, b54 = codes.WLAN_R12_BASE_Z81, codes.WLAN_R12_BASE
    assert ((b81 >= 0).sum(0) == (b54 >= 0).sum(0)).all() and (b81 >= 0).sum() == 86
    assert list(b81[[0, 6, 11], 12]) == [1, 0, 1] and (b81[:, 12][[1, 2, 3, 4, 5, 7, 8, 9, 10]] < 0).all()
    H = codes.wlan_80211n(81).toarray()
    assert (H[:, 1296:] != codes.wlan_80211n(81, base=b54).toarray()[:, 1296:]).sum() == 0  # same parity part
    overlap = H @ H.T
    np.fill_diagonal(overlap, 0)
    assert overlap.max() <= 1  # two checks share at most one variable: no 4-cycles
def test_table_lengths_follow_reference_layout():
    # Discrete_Density_Evolution.py:92-95 / :120-122 for the DVB-S2 profile (SURVEY §8 LUT lengths)
    assert tables.cn_lut_len(16, 16, 7, 50) == 256 + 4 * 256 + 49 * 5 * 256
    assert tables.vn_lut_len(16, 16, 8, 50) == 50 * (256 + 7 * 256)
    tb = tables.random_tables(16, 16, 7, 8, 50, seed=1)
    tb.check()
    assert tb.match_cn.size == 50 * 7 * 16 and tb.match_vn.size == 50 * 8 * 16
    bad = tables.random_tables(16, 16, 7, 8, 5)
    bad.cn[3] = 16
    with pytest.raises(ValueError):
        bad.check()


def test_channel_quantizer_contract():
    q = UniformQuantizer(sigma2_from_ebn0(1.0, 0.5), 16)
    L = q.output_LLRs
    assert np.all(np.diff(L) > 0)                  # clusters ordered by LLR
    np.testing.assert_allclose(L, -L[::-1], atol=1e-9)   # symmetric
    assert np.all(L[:8] < 0) and np.all(L[8:] > 0)  # cluster < T/2 <=> bit 1
    t = q.sample_all_zero(1000, 64, np.random.default_rng(0))
    assert t.min() >= 0 and t.max() <= 15
    emp = np.bincount(t.ravel(), minlength=16) / t.size
    np.testing.assert_allclose(emp, q.p_t_given_x0, atol=5e-3)
    assert sigma2_from_ebn0(0.0, 0.5) == pytest.approx(1.0)


def test_dropin_classes_setup_without_gpu(wlan_H, dvb_H):
    """Constructors are host-only and expose the reference's attributes; decoding without a
    GPU fails loudly (no CPU fallback)."""
    import torch
    from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular
    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import \
        Discrete_LDPC_Decoder_class_irregular
    g = graph.build_graph(dvb_H)
    tb = tables.random_tables(16, 16, 7, 8, 10)
    d = Discrete_LDPC_Decoder_class_irregular(dvb_H, 10, 16, 16, tb.cn, tb.vn, tb.match_cn, tb.match_vn, 2)
    assert d.data_len == 32399 and d.R_c == 0.4999999999999999
    assert d.d_c_max == 7 and d.d_v_max == 8 and d.N_v == 64800
    np.testing.assert_array_equal(d.target_memory_cells_varnodes, g.tgt_vn)
    bp = BeliefPropagationDecoderClassIrregular(wlan_H, 10, 16, 4)
    assert bp.data_len == 648
    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    with pytest.raises(RuntimeError, match="no HIP device"):
        d.decode_OpenCL(np.zeros((64800, 2), dtype=np.int32))
    with pytest.raises(RuntimeError, match="no HIP device"):
        bp.decode_OpenCL_belief_propagation(np.zeros((1296, 4)))


def test_decode_kernels_have_no_private_segment(lib):
    """Every decode kernel of the built library runs without scratch (no register spill, no item
    passed through private memory): the code object's metadata says private_segment_fixed_size 0.
    ibl_ib_create / ibl_float_create check the same at run time (hipFuncGetAttributes) and refuse
    a build that violates it (DESIGN.md "Private segment")."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import subprocess
    import tempfile
    from kstats import code_objects
    seen = {}
    for co in code_objects(lib.LIB_PATH):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name],
                                 capture_output=True, text=True).stdout
        for blk in re.split(r"\n\s+- \.", txt):
            m = re.search(r"\.name:\s+(\S+)", blk)
            p = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
            if m and p and re.search(r"(ib|fl)_(cn|vn|dec|fused)", m.group(1)):
                seen[m.group(1)] = int(p.group(1))
    assert len(seen) >= 20, seen
    assert {k: v for k, v in seen.items() if v} == {}


def test_generated_schedules_are_current():
    """csrc/ib_sched.inc is exactly what tools/gen_sched.py emits with the parameters named in its first
    line (a hand edit or a stale regeneration fails here, not only in the GPU bit-exact tests)."""
    import subprocess
    inc = os.path.join(ROOT, "informationbottleneckdecodingldpc_amd", "csrc", "ib_sched.inc")
    with open(inc) as fh:
        text = fh.read()
    first = text.splitlines()[0]
    assert first.startswith("// GENERATED by tools/gen_sched.py")
    args = first[len("// GENERATED by tools/gen_sched.py"):].split("--")[0].split()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_sched.py"), *args],
                       capture_output=True, text=True, check=True)
    assert r.stdout == text


def test_device_graph_lives_with_its_decoder(monkeypatch, wlan_H):
    """the device copy of a decoder's edge arrays is held by the decoder, not by a module
    cache, so 100 decoders constructed and dropped (one per Eb/N0 point, say) leave no device graph alive."""
    import gc
    import weakref

    import torch
    from informationbottleneckdecodingldpc_amd import _dropin

    class FakeGraph:
        def __init__(self, edges, dev):
            self.edges = edges

    monkeypatch.setattr(_dropin, "Graph", FakeGraph)
    refs = []
    for _ in range(100):
        d = _dropin.CodeMixin()
        d._init_code(wlan_H)
        g = d._graph_on(torch.device("cuda", 0))
        assert d._graph_on(torch.device("cuda", 0)) is g          # reused per decoder and device
        refs.append(weakref.ref(g))
        del d, g
    gc.collect()
    assert not hasattr(_dropin, "_GRAPH_CACHE")
    assert sum(r() is not None for r in refs) == 0


@pytest.fixture(scope="module")
def plan_check(tmp_path_factory):
    """tests/asan/plan_check.cpp with the product's host planning code (csrc/plan.h) under AddressSanitizer and
    UndefinedBehaviorSanitizer (host code only; GPU sanitizers are not available on the pool)."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not found")
    exe = str(tmp_path_factory.mktemp("asan") / "plan_check")
    subprocess.run([gxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "informationbottleneckdecodingldpc_amd", "csrc"),
                    os.path.join(ROOT, "tests", "asan", "plan_check.cpp"), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("name", ["dvb", "wlan", "wlan1944", "reg", "reg8000", "mixed", "singular"])
def test_host_planning_under_sanitizers(plan_check, tmp_path, name, dvb_H, wlan_H, reg_H):
    """the host planning the C ABI runs at create — map_node_connections, work orders and
    small-batch tasks, the float degree-2 fold plan, the fused task tables (both variable orders) and the encoder
    plan — built with ASan + UBSan, on every code the tests and benches use: no sanitizer report, every invariant
    holds, and the plans are the ones the GPU tests rely on (DVB-S2: 32,399 folded variables, a bidiagonal forward
    substitution)."""
    import json
    import subprocess
    from tests._codes import mixed_code
    H = {"dvb": lambda: dvb_H, "wlan": lambda: wlan_H, "wlan1944": lambda: codes.wlan_80211n(81),
         "reg": lambda: reg_H, "reg8000": lambda: codes.regular_code(8000, 3, 6, seed=0),
         "mixed": lambda: mixed_code(np.arange(2, 17), np.arange(1, 17), 600, seed=15),
         "singular": lambda: codes.regular_code(504, 3, 6, seed=0)}[name]()
    A = codes.canonical_csr(H)
    f = tmp_path / "g.bin"
    with open(f, "wb") as fh:
        np.array([A.shape[1], A.shape[0]], np.int32).tofile(fh)
        A.indptr.astype(np.int32).tofile(fh)
        A.indices.astype(np.int32).tofile(fh)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([plan_check, str(f)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    out = json.loads(r.stdout)
    g = graph.build_graph(H)
    assert (out["n_v"], out["n_c"], out["n_e"]) == (g.n_v, g.n_c, g.n_e) and out["failures"] == 0
    if name == "dvb":
        assert out["folded"] == 32399 and out["algo"] == "Forward Substitution" and out["chain"] == 1
    if name == "singular":
        assert out["encoder_rc"] == -2             # the reference prints "Not invertible Matrix"
    if name in ("wlan", "wlan1944"):
        assert out["encoder_rc"] == 0
