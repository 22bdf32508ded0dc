"""GPU: the device channel generator (ibl_channel_sample) against the oracle — bit-exact cluster ids
for every output type, mirrored codeword bits, ragged shapes and counter offsets — its distribution
at the DVB-S2 bench size, and the drop-in quantiser + BER driver end to end on the HIP decoders."""
import numpy as np
import pytest
import torch

from informationbottleneckdecodingldpc_amd import codes, engine, graph, tables
from informationbottleneckdecodingldpc_amd.awgn_quantizer import AWGN_Channel_Quantizer
from informationbottleneckdecodingldpc_amd.ber import BERConfig, run_ber
from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _q(ebn0=0.6, T=16):
    return UniformQuantizer(sigma2_from_ebn0(ebn0, 0.5), T=T)


@pytest.mark.parametrize("dtype", [torch.uint8, torch.int32, torch.float32, torch.float64])
@pytest.mark.parametrize("n,B,seed,offset", [(7, 5, 0, 0), (64, 1, 3, 17), (33, 1027, 2 ** 40 + 1, 2 ** 64 - 5),
                                              (1, 4, 9, 0)])
def test_channel_sample_equals_oracle(dtype, n, B, seed, offset):
    q = _q()
    out = torch.full((n, B), 99, dtype=dtype, device=DEV)
    engine.channel_sample(out, q.cdf_t_given_x_equals_zero, seed, offset, llr=q.output_LLRs)
    torch.cuda.synchronize()
    t = oracle.channel_sample(q.cdf_t_given_x_equals_zero, seed, offset, n, B)
    got = out.cpu().numpy()
    if dtype in (torch.uint8, torch.int32):
        assert np.array_equal(got.astype(np.int32), t)
    else:
        want = q.output_LLRs[t].astype(np.float32 if dtype == torch.float32 else np.float64)
        assert np.array_equal(got, want)


@pytest.mark.parametrize("T", [2, 8, 32, 64])
def test_channel_sample_bits_and_alphabets(T):
    q = _q(1.0, T)
    n, B = 40, 77
    bits = np.random.default_rng(T).integers(0, 2, (n, B)).astype(np.uint8)
    out = torch.empty((n, B), dtype=torch.int32, device=DEV)
    engine.channel_sample(out, q.cdf_t_given_x_equals_zero, 5, 11, bits=torch.from_numpy(bits).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), oracle.channel_sample(q.cdf_t_given_x_equals_zero, 5, 11, n, B, bits))


@pytest.mark.parametrize("case", ["clustered", "ties", "unsorted", "nan"])
def test_channel_sample_cdf_shapes(case):
    """The binned inversion (sorted thresholds: one table load per sample, compares only in bins holding
    thresholds) and its fallback (unsorted or NaN CDFs: T compares) equal the oracle's direct count: thresholds
    packed into one bin (many compares in it), repeated values, a decreasing entry, a NaN entry."""
    T = 16
    if case == "clustered":
        cdf = np.concatenate([[0.0], 0.5 + 1e-7 * np.arange(T - 1), [1.0]])
    elif case == "ties":
        cdf = np.concatenate([[0.0], np.repeat([0.25, 0.5, 0.75], 5), [1.0]])
    else:
        cdf = np.linspace(0.0, 1.0, T + 1)
        cdf[7] = 0.2 if case == "unsorted" else np.nan
    n, B = 64, 515
    out = torch.empty((n, B), dtype=torch.int32, device=DEV)
    engine.channel_sample(out, cdf, 12, 3)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), oracle.channel_sample(cdf, 12, 3, n, B))


def test_channel_batches_continue_the_stream():
    q = _q()
    cdf = q.cdf_t_given_x_equals_zero
    n, B = 10, 300
    full = torch.empty((2 * n, B), dtype=torch.uint8, device=DEV)
    halves = [torch.empty((n, B), dtype=torch.uint8, device=DEV) for _ in range(2)]
    engine.channel_sample(full, cdf, 1, 0)
    engine.channel_sample(halves[0], cdf, 1, 0)
    engine.channel_sample(halves[1], cdf, 1, engine.philox_blocks(n, B))
    assert torch.equal(torch.cat(halves), full)


def test_channel_distribution_at_bench_size():
    """64800 x 8192 samples: empirical cluster frequencies match p(t | x=0) (5-sigma binomial)."""
    q = _q(0.6)
    out = torch.empty((64800, 8192), dtype=torch.uint8, device=DEV)
    engine.channel_sample(out, q.cdf_t_given_x_equals_zero, 123, 0)
    counts = torch.bincount(out.view(-1).long(), minlength=16).cpu().numpy().astype(np.float64)
    total = out.numel()
    p = q.p_t_given_x0
    sd = np.sqrt(total * p * (1 - p))
    assert np.all(np.abs(counts - total * p) <= 5 * sd + 1), (counts / total, p)
    # the matching host stream gives the same first row
    assert np.array_equal(out[0].cpu().numpy().astype(np.int32),
                          oracle.channel_sample(q.cdf_t_given_x_equals_zero, 123, 0, 1, 8192)[0])


def test_dropin_quantizer_device_paths():
    s2 = sigma2_from_ebn0(0.6, 0.5)
    q = AWGN_Channel_Quantizer(s2, 3, 16, 2000, seed=7)
    q.init_OpenCL_quanti(100, 33, return_buffer_only=True)
    a = q.quantize_direct_OpenCL(100, 33)
    assert a.dtype == torch.int32 and a.shape == (100, 33) and a.device.type == "cuda"
    want = oracle.channel_sample(q.cdf_t_given_x_equals_zero, 7, 0, 100, 33)
    assert np.array_equal(a.cpu().numpy(), want)
    llr = q.quantize_direct_OpenCL_LLR(100, 33)
    t2 = oracle.channel_sample(q.cdf_t_given_x_equals_zero, 7, engine.philox_blocks(100, 33), 100, 33)
    assert llr.dtype == torch.float64 and np.array_equal(llr.cpu().numpy(), q.output_LLRs[t2])
    q.return_buffer_only = False
    h = q.quantize_direct_OpenCL(100, 33, dtype=torch.uint8)
    assert isinstance(h, np.ndarray) and h.dtype == np.uint8


def test_ber_driver_ib_wlan_end_to_end():
    """IB decoder on WLAN with LLR-derived tables (tables.llr_tables): device channel -> decode ->
    error count; at 5 dB the decoder corrects everything, at -2 dB it does not."""
    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import \
        Discrete_LDPC_Decoder_class_irregular
    H = codes.wlan_80211n()
    g = graph.build_graph(H)
    imax = 20
    qz = _q(5.0)
    tb = tables.llr_tables(qz.output_LLRs, g.d_c_max, g.d_v_max, imax)
    dec = Discrete_LDPC_Decoder_class_irregular(H, imax, 16, 16, tb.cn, tb.vn, tb.match_cn, tb.match_vn, 256,
                                                match="true")
    cfg = BERConfig(EbN0_dB_start=5.0, EbN0_dB_max_value=5.0, min_errors=1, msg_at_time=256, max_blocks=2048,
                    seed=3)
    r = run_ber(dec, cfg)
    assert r.blocks == [2048] and r.errors == [0.0] and r.BER_vector[0] == 0.0
    cfg2 = BERConfig(EbN0_dB_start=-2.0, EbN0_dB_max_value=-2.0, min_errors=1000, msg_at_time=256, seed=3)
    r2 = run_ber(dec, cfg2)
    assert r2.errors[0] >= 1000 and 1e-3 < r2.BER_vector[0] < 0.5


def test_ber_driver_minsum_llr_input():
    from informationbottleneckdecodingldpc_amd.min_sum_decoder_irreg import Min_Sum_Decoder_class_irregular
    H = codes.wlan_80211n()
    dec = Min_Sum_Decoder_class_irregular(H, 20, 16, 128)
    cfg = BERConfig(EbN0_dB_start=5.0, EbN0_dB_max_value=5.0, min_errors=1, msg_at_time=128, max_blocks=1024,
                    llr_dtype=torch.float32)
    r = run_ber(dec, cfg)
    assert r.blocks == [1024] and r.errors == [0.0]


@pytest.mark.parametrize("dtype", [torch.uint8, torch.int32, torch.float32, torch.float64])
def test_channel_sample_row_stride(dtype):
    """ibl_channel_sample with a row stride ld > B (the C ABI's general case; the round-6 kernel's per-block row
    split): the [n][B] window equals the oracle, the padding columns stay untouched."""
    from informationbottleneckdecodingldpc_amd import _lib
    q = _q()
    n, B, ld = 9, 13, 16
    buf = torch.full((n, ld), 77, dtype=dtype, device=DEV)
    cdf = np.ascontiguousarray(q.cdf_t_given_x_equals_zero, np.float64)
    llr = np.ascontiguousarray(q.output_LLRs, np.float64)
    _lib.check(_lib.load().ibl_channel_sample(cdf, 16, llr.ctypes.data, 4, 21, n, B, None, buf.data_ptr(),
                                              engine._DT_ANY[dtype], ld, engine._stream_ptr(buf.device)),
               "ibl_channel_sample")
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    t = oracle.channel_sample(q.cdf_t_given_x_equals_zero, 4, 21, n, B)
    want = t if dtype in (torch.uint8, torch.int32) else q.output_LLRs[t].astype(got.dtype)
    assert np.array_equal(got[:, :B].astype(want.dtype), want)
    assert np.all(got[:, B:] == 77)


@pytest.mark.parametrize("dtype", [torch.uint8, torch.int32, torch.float32, torch.float64])
@pytest.mark.parametrize("B,ld", [(96, 96), (4096, 4096), (48, 64), (77, 77)])
def test_counters_vector_and_strided(dtype, B, ld):
    """ibl_count_below / ibl_count_errors (round 6: one 16-byte word per lane when rows, stride and pointer allow it,
    else one element; row stride ld >= B) equal numpy on the [rows][B] window."""
    from informationbottleneckdecodingldpc_amd import _lib
    rng = np.random.default_rng(B + ld)
    n, rows = 37, 29
    full = rng.integers(0, 16, (n, ld)) if dtype in (torch.uint8, torch.int32) else rng.normal(size=(n, ld))
    bits = rng.integers(0, 2, (n, ld)).astype(np.uint8)
    thr = 8 if dtype in (torch.uint8, torch.int32) else 0.0
    x = torch.from_numpy(full).to(dtype).to(DEV)
    bt = torch.from_numpy(bits).to(DEV)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    L = _lib.load()
    s = engine._stream_ptr(x.device)
    _lib.check(L.ibl_count_below(x.data_ptr(), engine._DT_ANY[dtype], rows, B, ld, float(thr), cnt.data_ptr(), s), "cb")
    assert int(cnt.item()) == int((full[:rows, :B] < thr).sum())
    _lib.check(L.ibl_count_errors(x.data_ptr(), engine._DT_ANY[dtype], rows, B, ld, float(thr), bt.data_ptr(), ld,
                                  cnt.data_ptr(), s), "ce")
    assert int(cnt.item()) == int(((full[:rows, :B] < thr) != (bits[:rows, :B] != 0)).sum())
    # half thresholds on integer outputs: v < 7.5 <=> v < 8
    if dtype in (torch.uint8, torch.int32):
        _lib.check(L.ibl_count_below(x.data_ptr(), engine._DT_ANY[dtype], rows, B, ld, 7.5, cnt.data_ptr(), s), "cb")
        assert int(cnt.item()) == int((full[:rows, :B] < 7.5).sum())
