"""Benchmark: batched DVB-S2 IB-LUT decoding on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch-per-gpu B] [--imax I]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)
    python bench.py --config C1|C2|C3|C5                   (BASELINE.json's other configs)

Default = BASELINE config C4 (the headline metric). The other presets measure the remaining
configs of BASELINE.json: C1 regular (3,6) N=8000 IB T=16 i_max=10, 1000 codewords (the reference's
CPU case: its numpy decode_on_host, restated in oracle/host_numpy.py, is the cpu_baseline, one
process per host core, next to the GPU decoding the same 1000 codewords); C2 regular (3,6) N=8000
IB T=16 i_max=50, 65536 codewords; C3 WLAN 802.11n N=1944 (the standard's Z=81 table) min-sum fp32
i_max=50, 262144 codewords; C5 DVB-S2 BP fp32 i_max=100, 8192 codewords per GPU. The regular
configs run without matching (the reference's regular class has none).

A "step" = one decode call of B codewords per GPU (DVB-S2-structured N=64800 R=1/2 code,
T=16 lookup tables with matching, i_max=50 fixed iterations — early stop off, as the roofline
plan in BASELINE.md prescribes). Inputs are generated on the device before the timed region
(all-zero codeword, BPSK, AWGN at Eb/N0 = 0.6 dB, 16-cluster quantiser). Work per GPU is fixed
as N grows (weak scaling); codeword ranges are disjoint per rank and no collective runs inside
the timed region.

Rank 0 prints one JSON line with the whole-job codewords/s, the algorithmic HBM GB/s, the
roofline of the dominant kernel (HIP-event timed per launch in the last step of the timed region — events
around every launch of every step cost ~1.3 % of a C4 step, round 6; priced at the
bytes the kernel actually moves: 4-bit messages on the IB fast path, LDS bytes for the fused on-chip
float kernel) and the CPU baseline on a bounded sample: the reference's numpy host path
(restated) where the reference has one (regular IB: C1, C2), else the C oracle (a port of the
reference's OpenCL kernels).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
CH_SEED = 2              # Philox key of the synthetic channel ("seed 2, keyed by global codeword index")


def parse(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--batch-per-gpu", type=int, default=8192)
    p.add_argument("--imax", type=int, default=50)
    p.add_argument("--ebn0", type=float, default=None, help="Eb/N0 in dB (default 0.6; 1.0 with --early-stop)")
    p.add_argument("--kind", choices=["ib", "minsum", "bp"], default="ib")
    p.add_argument("--code", choices=["dvbs2", "regular", "wlan"], default="dvbs2")
    p.add_argument("--config", choices=["C1", "C2", "C3", "C4", "C5"], default=None,
                   help="BASELINE.json config preset (sets --code/--kind/--imax/--batch-per-gpu)")
    p.add_argument("--no-match", action="store_true")
    p.add_argument("--path", "--float-path", dest="path", choices=["auto", "passes", "fused"], default="auto",
                   help="fused on-chip kernel when the code fits in LDS (auto), or per-pass launches")
    p.add_argument("--cpu-sample", type=int, default=100000, help="cap on the CPU-baseline sample (sized to ~12 s of CPU work)")
    p.add_argument("--cpu-procs", type=int, default=0, help="CPU-baseline processes / oracle threads (0 = this job's CPU share, bench.cpu_share())")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-kernel-events", action="store_true",
                   help="diagnostics: no HIP events around the launches (value without their gaps; no roofline timing)")
    p.add_argument("--early-stop", action="store_true",
                   help="batch-global early stop on (SURVEY §8(d)'s second line: at 1.0 dB unless --ebn0 is given); "
                        "IB decoders use density-evolution tables (tables.de_tables, designed at 0.75 dB) so the batch can converge")
    p.add_argument("--sub-batch", type=int, default=0,
                   help="IB only: decode the batch as sequential sub-batches of this many codewords (one decoder sized "
                        "for the sub-batch: its working set can stay in the 256-MiB Infinity Cache across passes)")
    p.add_argument("--batch-offset", type=int, default=0,
                   help="global batch index of rank 0's batch: rank r decodes global batch offset + r, whose channel "
                        "is Philox key 2 at counter (offset + r) * philox_blocks(N, B) (SURVEY H9)")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    a = p.parse_args(argv)
    presets = {"C1": ("regular", "ib", 10, 1000), "C2": ("regular", "ib", 50, 65536),
               "C3": ("wlan", "minsum", 50, 262144), "C4": ("dvbs2", "ib", 50, 8192), "C5": ("dvbs2", "bp", 100, 8192)}
    if a.config:
        a.code, a.kind, a.imax, B = presets[a.config]
        if "--batch-per-gpu" not in argv:
            a.batch_per_gpu = B
        if a.config in ("C1", "C2"):
            a.no_match = True      # Discrete_LDPC_Decoder_class (regular) has no matching step
    if a.ebn0 is None:
        a.ebn0 = 1.0 if a.early_stop else 0.6
    return a


CODES = {"dvbs2": ("DVB-S2 N=64800 R=1/2", "DVB-S2-structured R=1/2 code (EN 302 307 profile, synthetic addresses)"),
         "regular": ("regular (3,6) N=8000", "seeded (3,6)-regular N=8000 code (stands in for MacKay 8000.4000.3.483)"),
         "wlan": ("WLAN 802.11n N=1944 R=1/2", "802.11n R=1/2 Z=81 prototype (IEEE 802.11-2012 Table F.2)")}


def make_code(name):
    from informationbottleneckdecodingldpc_amd import codes
    if name == "dvbs2":
        return codes.dvbs2_structured(seed=0)
    if name == "regular":
        return codes.regular_code(8000, 3, 6, seed=0)
    return codes.wlan_80211n(81)


def bytes_per_cw(n_e: int, n_v: int, imax: int, w: int) -> int:
    """SURVEY §8(d)'s fixed reporting width: i_max·(4·E·w_m + N·w_c) + N·(w_c + w_o) — the u8-equivalent
    figure (reported as *_u8_equivalent; the 4-bit and fused paths never move these bytes)."""
    return imax * (4 * n_e * w + n_v * w) + n_v * (w + w)


def moved_bytes_per_cw(n_e: int, n_v: int, imax: int, path: str, ws: float, w_in: int, w_out: int,
                       w_stage: float = 1, folded: int = 0) -> float:
    """HBM bytes one codeword's decode moves at the widths the kernels store (fixed iterations).

    per-pass IB (ws < 4): stage (read N·w_in, write N·ws); check pass 0 (gathers the staged channel per edge,
    writes E); i_max−1 loop iterations of variable pass (read E+N, write E) + check pass (read E, write E);
    decision (read E+N, write N·w_out) — messages at ws bytes.
    per-pass float (ws >= 4): stage; send (read N, write E); i_max−1 check passes (read E, write E; the
    i_max−2 that fold `folded` degree-2 variables also read their 2 channel rows); i_max−2 variable passes
    (the last iteration's feeds no output and is not run) over the unfolded variables (read E'+N', write E',
    E' = E − 2·folded, N' = N − folded); decision.
    fused ("fused"): channel in (N·w_in), the transposed staging copy (N·w_stage written and read: u8 for IB,
    the float width for min-sum / BP), output out (N·w_out); the messages never leave LDS."""
    E, N = n_e, n_v
    if path == "fused":
        return N * w_in + 2 * N * w_stage + N * w_out
    if ws < 4:
        return (N * w_in + N * ws + 2 * E * ws
                + (imax - 1) * (4 * E + N) * ws + (E + N) * ws + N * w_out)
    nf = folded
    loop = 0
    if imax >= 2:
        loop = (imax - 1) * 2 * E + (imax - 2) * (2 * nf + 2 * (E - 2 * nf) + (N - nf))
    return N * w_in + N * ws + (E + N) * ws + loop * ws + (E + N) * ws + N * w_out


LDS_CLK_GHZ = 2.4          # MI355X max engine clock (MI355X_MICROARCH.md chip table)
NUM_CUS = 256


def _pmc_traffic(path, kind, kname, B, fmt):
    """Per-launch HBM bytes of `kname` from the committed rocprofv3 PMC summary, when it was measured
    on the same kernel, batch and message format (else None)."""
    if not os.path.exists(path):
        return None
    try:
        with open(path) as fh:
            ent = json.load(fh).get(kind, {}).get(kname)
        if ent and int(ent.get("batch", -1)) == B and ent.get("format") == fmt:
            return ent.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def roofline(a, g, n_v, B, I, w, ws, fmt, match, fused, cn_avg, vn_avg, cn_ms, vn_ms, cn_n, vn_n, dec, folded=0,
             small=False):
    """Roofline of the dominant kernel, priced at the bytes it actually moves.

    Per-pass kernels (HBM-bound by design): check pass reads E message rows and writes E; variable
    pass reads E rows + N channel rows and writes E (SURVEY §8(d) per-unit figures), x B codewords,
    at the stored width (u4 fast path, u8 generic, fp32 float). The u8-equivalent of SURVEY §8(d)'s
    fixed reporting width is kept as a secondary field. The fused on-chip float kernel keeps every
    message in LDS: its roofline is the LDS's (16-B slot reads at 256 B/clk/CU, 16-B slot writes at
    79 B/clk/CU, MI355X_MICROARCH.md §LDS), with its HBM bytes (channel in, APP out) reported beside."""
    cn_bytes_u8 = 2 * g.n_e * w * B
    vn_bytes_u8 = (2 * g.n_e * w + n_v * w) * B
    if folded and fmt == "f32":
        # degree-2 fold (float per-pass): the variable pass covers E - 2 nf edges and N - nf variables; the
        # check passes that fold (all but the last of cn_n) also read 2 channel rows per folded variable
        vn_bytes_u8 = (2 * (g.n_e - 2 * folded) + (n_v - folded)) * w * B
        fold_frac = max(cn_n - 1, 0) / max(cn_n, 1)
        cn_bytes_u8 = int(round((2 * g.n_e + 2 * folded * fold_frac) * w * B))

    def cn_lk(d):     # table lookups of one check of degree d per codeword (prefix sharing, matching composed)
        return (2 if match else 0) if d == 2 else (d - 2) + d * (d - 1) // 2 - 1

    def vn_lk(d):
        return 0 if d == 1 else (d - 1) + d * (d - 1) // 2
    if fused and a.kind == "ib":
        # fused IB kernel: per 8-codeword group and iteration every check reads and writes its d slot
        # dwords and makes 8*cn_lk(d) ds_read_u8 lookups, every variable likewise; LDS cycles per
        # wave-instruction (64 lanes): ds_read_u8 / ds_read_b32 2, ds_write_b32 4 (MI355X_MICROARCH.md
        # §LDS). achieved/peak = LDS bytes moved (a lookup moves 1 B) over time / at this mix's rate.
        L = I - 1
        cd, vd = np.asarray(g.cn_deg, np.int64), np.asarray(g.vn_deg, np.int64)
        lk_cn = 8 * sum(cn_lk(int(d)) for d in cd)
        lk_vn = 8 * sum(vn_lk(int(d)) for d in vd)
        lk_dec = 8 * int(vd.sum())
        E = int(cd.sum())
        groups = -(-B // 8)
        # per group: send (E slot writes), L+1 CN passes, L VN passes, decision (E slot reads)
        rd_slots = (L + 1) * E + L * E + E
        wr_slots = E + (L + 1) * E + L * E
        lookups = (L + 1) * lk_cn + L * lk_vn + lk_dec
        cyc = groups * (rd_slots * 2 + wr_slots * 4 + lookups * 2) / 64.0        # LDS cycles (chip, summed)
        byts = groups * (4 * (rd_slots + wr_slots) + lookups)
        t = cn_avg * 1e-3
        peak = byts / cyc * NUM_CUS * LDS_CLK_GHZ if cyc else 0.0
        ach = byts / t / 1e9 if t > 0 else 0.0
        return {"bound": "lds", "kernel": "ib_fused", "achieved": round(ach, 1), "peak": round(peak, 1),
                "unit": "GB/s", "frac": round(ach / peak, 4) if peak else 0.0, "traffic": None,
                "bytes_per_launch": int(byts), "avg_launch_ms": round(cn_avg, 4),
                "lds_lookups_per_clk_per_cu": round(groups * lookups / t / (NUM_CUS * LDS_CLK_GHZ * 1e9), 2) if t > 0 else 0,
                "hbm": {"bytes_per_launch": 2 * n_v * B, "peak": HBM_PEAK_GBPS},
                "note": "fused on-chip IB decoder: 8 codewords per workgroup, 4-bit messages in LDS for all "
                        "iterations; LDS roofline at this kernel's mix of ds_read_u8 lookups and dword slot "
                        "reads/writes (MI355X_MICROARCH.md §LDS); lds_lookups_per_clk_per_cu against 32",
                "launches": {"fused": cn_n}}
    if fused:
        # one launch decodes the whole batch: L = imax-1 check passes, L-1 variable passes (16-B slots,
        # N codewords per slot), plus send (E+N slot writes) and the APP output (E+N slot reads)
        L = I - 1
        E = g.n_e
        slots_r = L * E + max(L - 1, 0) * (E + n_v) + (E + n_v)
        slots_w = (E + n_v) + L * E + max(L - 1, 0) * E
        groups = -(-B // 4)
        rd, wr = 16 * slots_r * groups, 16 * slots_w * groups
        t = cn_avg * 1e-3
        peak = (rd + wr) / (rd / 256 + wr / 79) * NUM_CUS * LDS_CLK_GHZ   # GB/s at the instruction mix
        ach = (rd + wr) / t / 1e9 if t > 0 else 0.0
        return {"bound": "lds", "kernel": "fl_fused", "achieved": round(ach, 1), "peak": round(peak, 1),
                "unit": "GB/s", "frac": round(ach / peak, 4), "traffic": None,
                "bytes_per_launch": rd + wr, "lds_read_bytes": rd, "lds_write_bytes": wr,
                "avg_launch_ms": round(cn_avg, 4),
                "hbm": {"bytes_per_launch": 2 * n_v * 4 * B, "achieved": round(2 * n_v * 4 * B / t / 1e9, 1) if t > 0 else 0.0,
                        "peak": HBM_PEAK_GBPS},
                "note": "fused on-chip decoder: messages of 4 codewords per workgroup stay in LDS for all "
                        "iterations; LDS roofline at this kernel's 16-B read/write mix (MI355X_MICROARCH.md §LDS)",
                "launches": {"fused": cn_n}}
    sfx = "_small" if small else ""
    if vn_ms >= cn_ms:
        kname = ("ib_vn_small" if small else "ib_vn_fast") if fmt == "u4" else ("ib_vn_gen" if a.kind == "ib" else "fl_vn" + sfx)
        kavg, ku8 = vn_avg, vn_bytes_u8
    else:
        kname = ("ib_cn_small" if small else "ib_cn_fast") if fmt == "u4" else ("ib_cn_gen" if a.kind == "ib" else "fl_cn" + sfx)
        kavg, ku8 = cn_avg, cn_bytes_u8
    kbytes = int(ku8 * ws / w)
    t = kavg * 1e-3
    ach = kbytes / t / 1e9 if t > 0 else 0.0
    roof = {"bound": "hbm", "kernel": kname, "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": _pmc_traffic(a.pmc, a.kind, kname, B, fmt),
            "bytes_per_launch": kbytes, "format": fmt, "avg_launch_ms": round(kavg, 4),
            "u8_equivalent": {"bytes_per_launch": ku8, "achieved": round(ku8 / t / 1e9, 1) if t > 0 else 0.0,
                              "note": "SURVEY §8(d)'s fixed u8 reporting width; not the bytes this kernel moves"}
            if fmt == "u4" else None,
            "launches": {"cn": cn_n, "vn": vn_n},
            "avg_ms": {"cn": round(cn_avg, 4), "vn": round(vn_avg, 4)}}
    if fmt == "f32":
        # both passes of the per-pass float path against HBM (bytes per launch at fp32)
        roof["passes"] = {k: {"bytes_per_launch": int(b * ws / w), "avg_launch_ms": round(t_, 4),
                              "achieved": round(b * ws / w / (t_ * 1e-3) / 1e9, 1) if t_ > 0 else 0.0,
                              "frac": round(b * ws / w / (t_ * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if t_ > 0 else 0.0}
                          for k, b, t_ in (("cn", cn_bytes_u8, cn_avg), ("vn", vn_bytes_u8, vn_avg))}
        if folded:
            roof["folded_degree2_variables"] = folded
    if fmt == "u4":
        # table lookups per codeword and pass of the fast path, per CU and clock at the max clock; the LDS
        # serves at most 32 conflict-free ds_read_u8 lanes/clk/CU
        lk = {"cn": int(sum(cn_lk(int(d)) for d in g.cn_deg)) * B, "vn": int(sum(vn_lk(int(d)) for d in g.vn_deg)) * B}
        avg = {"cn": cn_avg, "vn": vn_avg}
        roof["lds_lookups_per_clk_per_cu"] = {k: round(lk[k] / (avg[k] * 1e-3) / (NUM_CUS * LDS_CLK_GHZ * 1e9), 2)
                                              for k in lk if avg[k] > 0}
        roof["lds_lookups_per_clk_per_cu"]["ceiling"] = 32.0
        mc = measured_lookup_ceiling()
        if mc:
            roof["lds_lookups_per_clk_per_cu"]["measured_chain_rate"] = mc
    return roof


def measured_lookup_ceiling(path=os.path.join(ROOT, "profiles", "r03_ubench_lookup_rate.json")):
    """Highest LDS-only lookup rate (lookups/clk/CU at the nominal clock) that tools/ubench/lookup_rate.hip
    measured for dependent ds_read_u8 chains on the decoders' table layout (profiles/, JSON lines), or None."""
    try:
        with open(path) as fh:
            rows = [json.loads(l) for l in fh if l.strip()]
        rates = [r["lookups_per_clk_per_cu"] for r in rows if r.get("global_chains") == 0]
        return round(max(rates), 2) if rates else None
    except (OSError, ValueError, KeyError):
        return None


def aggregate_rate(B: int, steps: int, elapsed_local: float) -> dict:
    """Whole-job rate over the ranks of the process group: world·B·steps ÷ the slowest rank's timed region
    (max over ranks), plus what the group was (backend, world size) and the per-rank rates (min / max), so a
    multi-GPU record shows which backend and how many ranks produced it."""
    import torch.distributed as dist

    from informationbottleneckdecodingldpc_amd import distributed
    on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size() if on else 1
    mx = distributed.allreduce_max(elapsed_local)
    mn = -distributed.allreduce_max(-elapsed_local)
    return {"value": world * B * steps / mx, "elapsed_max_s": mx, "world_size": world,
            "backend": dist.get_backend() if on else "none",
            "per_rank_codewords_per_s": {"min": B * steps / mx, "max": B * steps / mn}}


def cpu_share() -> int:
    """CPUs this process may use: the affinity mask, capped by a cgroup v2 quota and by the job's
    OMP_NUM_THREADS (the GPU box grants one GPU's job a 16-CPU share of a many-core host and says so there;
    os.cpu_count() reports the whole host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
            if q != "max":
                n = min(n, max(1, -(-int(q) // int(p))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ---- numpy host baseline workers (spawned processes: they never touch the GPU)
_HOST = {}


def _host_init(arrs, Tc, T, imax, cn_lut, vn_lut, regular):
    import types
    from oracle.host_numpy import HostDecoder
    _HOST["dec"] = HostDecoder(types.SimpleNamespace(**arrs), Tc, T, imax, cn_lut, vn_lut, regular=regular)


def _host_ready(_):
    return os.getpid()


def _host_decode(cols):
    dec = _HOST["dec"]
    return np.stack([dec.decode(c) for c in cols], axis=1)


def numpy_host_baseline(g, tb, x_host, imax, regular, procs):
    """The reference's CPU decode path (decode_on_host, oracle/host_numpy.py): per-core rate measured
    in this process, aggregate rate with `procs` single-threaded worker processes (spawned, so they
    hold no GPU state) decoding the sample's codewords one per call."""
    import multiprocessing as mp
    from oracle.host_numpy import HostDecoder
    keys = ("n_v", "n_e", "cn_deg", "cn_start", "tgt_cn", "vn_deg", "vn_start", "tgt_vn")
    arrs = {k: getattr(g, k) for k in keys}
    dec = HostDecoder(g, tb.Tc, tb.T, imax, tb.cn, tb.vn, regular=regular)
    S = x_host.shape[1]
    k1 = max(1, min(S, 8))
    dec.decode(x_host[:, 0])
    t1 = time.perf_counter()
    for c in range(k1):
        dec.decode(x_host[:, c])
    per_core = k1 / (time.perf_counter() - t1)
    # the same path in the reference's own shape of work (masks rebuilt with np.kron / np.eye every pass,
    # [E][1] inboxes): per-core rate beside the shape-optimised one the workers run
    dec_f = HostDecoder(g, tb.Tc, tb.T, imax, tb.cn, tb.vn, regular=regular, faithful_shape=True)
    dec_f.decode(x_host[:, 0])
    t1 = time.perf_counter()
    for c in range(k1):
        dec_f.decode(x_host[:, c])
    per_core_faithful = k1 / (time.perf_counter() - t1)
    for v in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[v] = "1"
    ctx = mp.get_context("spawn")
    chunks = [[x_host[:, c] for c in range(i, S, procs)] for i in range(procs)]
    with ctx.Pool(procs, initializer=_host_init,
                  initargs=(arrs, tb.Tc, tb.T, imax, tb.cn, tb.vn, regular)) as pool:
        pool.map(_host_ready, range(procs), chunksize=1)
        t1 = time.perf_counter()
        parts = pool.map(_host_decode, chunks, chunksize=1)
        wall = time.perf_counter() - t1
    outs = np.zeros((g.n_v, S), dtype=np.int64)
    for i, p_ in enumerate(parts):
        if p_.size:
            outs[:, i::procs] = p_
    return outs, per_core, S / wall, wall, per_core_faithful


def cpu_baseline(a, g, arrays, I, B, match, src, out, code_name):
    """Bounded-sample CPU baseline on this box's host cores (reported beside the GPU, not a target)."""
    from informationbottleneckdecodingldpc_amd import tables
    from oracle import oracle
    host = (lambda S_: src[:, :S_].cpu().numpy().astype(np.int32 if a.kind == "ib" else np.float64))  # noqa: E731
    ncpu = os.cpu_count() or 1
    share = cpu_share()
    proj_note = (f"per_core x host_cpus ({ncpu}); projected, not measured: this job's CPU share is {share} "
                 f"(affinity / cgroup quota / OMP_NUM_THREADS), and the box runs at most that many workers")
    if a.kind == "ib" and a.code == "regular" and not match:
        # the reference's own CPU path: numpy decode_on_host (regular class), one codeword per call
        procs = a.cpu_procs or share
        tbh = tables.IBTables(16, 16, g.d_c_max, g.d_v_max, I, arrays["cn"], arrays["vn"], arrays["mc"], arrays["mv"])
        per_cw_s = 0.0028 * I                         # ~2.8 ms per (3,6) N=8000 iteration per core
        S = int(min(B, a.cpu_sample, max(procs, 30.0 / per_cw_s)))   # ~30 s of CPU work
        if a.config == "C1":
            S = min(B, a.cpu_sample, 1000)            # C1 IS 1000 codewords on the CPU path
        x = host(S)
        ref, per_core, agg, wall, per_core_f = numpy_host_baseline(g, tbh, x, I, True, procs)
        same = bool(np.array_equal(ref, out[:, :S].cpu().numpy().astype(np.int64)))
        return {"value": round(agg, 3), "unit": "codewords/s", "cores": procs, "kind": "port",
                "per_core": round(per_core, 3), "per_core_faithful_shape": round(per_core_f, 3),
                "cpu_model": _cpu_model(), "host_cpus": ncpu, "cpu_share": share,
                "all_cores_projected": {"value": round(per_core * ncpu, 3), "note": proj_note},
                "sample": f"{S} of the benchmark's codewords, {code_name}, i_max={I}, no matching, fixed iterations; "
                          f"the reference's numpy decode_on_host (Discrete_LDPC_decoder_class, restated in "
                          f"oracle/host_numpy.py, bit-identical to the reference's outputs), one codeword per call, "
                          f"{procs} single-threaded processes, {wall:.1f} s wall; outputs equal GPU: {same}. The "
                          f"timed restatement is shape-optimised (the 'others' masks built once per degree, flat "
                          f"inboxes); per_core_faithful_shape is the same path with the reference's per-pass "
                          f"np.kron/np.eye masks and [E][1] inboxes (slower, so value errs high)"}
    nthreads = a.cpu_procs or share
    # bounded sample: a 16-codeword calibration run sizes the measured sample to ~12 s of CPU work
    if a.kind == "ib":
        tbh = tables.IBTables(16, 16, g.d_c_max, g.d_v_max, I, arrays["cn"], arrays["vn"], arrays["mc"], arrays["mv"])
        dec_cpu = lambda x, nt=nthreads: oracle.ib_decode(g, tbh, x, match=match, early_stop=False, nthreads=nt)  # noqa: E731
    elif a.kind == "minsum":
        # fp32 min-sum restated in IEEE single (oracle/float_oracle.inc): the same arithmetic as the GPU
        dec_cpu = lambda x, nt=nthreads: oracle.float32_decode(g, I, x.astype(np.float32), nthreads=nt)  # noqa: E731
    else:
        dec_cpu = lambda x, nt=nthreads: oracle.float_decode(g, 1, I, x, early_stop=False, nthreads=nt)  # noqa: E731
    S0 = min(16, B)
    t1 = time.perf_counter()
    dec_cpu(host(S0))
    cal = time.perf_counter() - t1
    # one thread: the per-core rate (about 2 s of work)
    S1 = int(max(1, min(S0, 2.0 * S0 / max(cal * nthreads, 1e-3))))
    x1 = host(S1)
    t1 = time.perf_counter()
    dec_cpu(x1, 1)
    per_core = S1 / (time.perf_counter() - t1)
    S = int(max(S0, min(B, a.cpu_sample, S0 * 12.0 / max(cal, 1e-3))))
    x_cpu = host(S)
    t1 = time.perf_counter()
    ref = dec_cpu(x_cpu)
    cpu_s = time.perf_counter() - t1
    if a.kind == "ib":
        same = bool(np.array_equal(ref, out[:, :S].cpu().numpy().astype(np.int32)))
        what = (f"oracle/ib_oracle.c (C+OpenMP restatement of the reference OpenCL kernels; the reference's "
                f"own numpy host path cannot decode this code or has no matching); outputs equal GPU: {same}")
    elif a.kind == "minsum":
        same = bool(np.array_equal(ref, out[:, :S].cpu().numpy()))
        what = (f"oracle/ib_oracle.c fp32 restatement of kernels_min_and_BP.cl's min-sum (the reference's float "
                f"host paths are broken, SURVEY App. C3); APP LLRs equal GPU bit for bit: {same}")
    else:
        o = out[:, :S].cpu().numpy().astype(np.float64)
        tol = 1e-5 * np.maximum(np.abs(o), np.abs(ref)) + 1e-4
        within = float(np.mean(np.abs(o - ref) <= tol))
        agree = float(np.mean((ref < 0) == (o < 0)))
        what = (f"oracle/ib_oracle.c fp64 restatement of kernels_min_and_BP.cl (the reference's float host "
                f"paths are broken, SURVEY App. C3); GPU fp32 APP LLRs within 1e-5 rel + 1e-4: {within:.6f}, "
                f"hard decisions equal: {agree:.6f}")
    return {"value": round(S / cpu_s, 3), "unit": "codewords/s", "cores": nthreads, "kind": "port",
            "per_core": round(per_core, 4), "cpu_model": _cpu_model(), "host_cpus": ncpu, "cpu_share": share,
            "all_cores_projected": {"value": round(per_core * ncpu, 3), "note": proj_note},
            "sample": f"{S} of the benchmark's codewords, {code_name}, i_max={I}, fixed iterations; {what}; "
                      f"{cpu_s:.1f} s wall"}


def setup_arrays(a):
    """Rank 0's setup payload: the code's canonical CSR and random T=16 tables (seed 1) with matching vectors."""
    from informationbottleneckdecodingldpc_amd import graph, tables
    g0 = graph.build_graph(make_code(a.code))
    tb0 = tables.random_tables(16, 16, g0.d_c_max, g0.d_v_max, a.imax, seed=1)
    return dict(indptr=g0.csr_indptr, cols=g0.csr_cols, shape=np.array([g0.n_c, g0.n_v]),
                cn=tb0.cn, vn=tb0.vn, mc=tb0.match_cn, mv=tb0.match_vn)


def graph_of(arrays):
    """Host edge graph of the broadcast CSR."""
    import scipy.sparse as sp

    from informationbottleneckdecodingldpc_amd import graph
    n_c, n_v = (int(x) for x in arrays["shape"])
    H = sp.csr_matrix((np.ones(arrays["cols"].size), arrays["cols"], arrays["indptr"]), shape=(n_c, n_v))
    return graph.build_graph(H)


def build_decoder(a, G, g, arrays, q, B):
    """The decoder a bench run times, from the parsed arguments `a` (the C1-C5 presets), the device graph G,
    the host graph g, rank 0's broadcast arrays (H and the random tables) and the channel quantiser q.
    Returns (decoder, match). tests/test_gpu_bench_paths.py builds every config's decoder through this, so
    the oracle tests run exactly the kernel path each bench line times."""
    import torch

    from informationbottleneckdecodingldpc_amd import engine, tables
    from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0
    I, match = a.imax, not a.no_match
    if a.kind == "ib":
        if a.early_stop:
            # tables that decode (so the batch can converge and stop): discrete density evolution at 0.75 dB, the
            # design point of the DVB-S2 curves in profiles/r06_dvbs2_ber_curves.json (round 6; was llr_tables)
            qd = UniformQuantizer(sigma2_from_ebn0(0.75, g.R_c), 16)
            rho, lam = tables.edge_degree_distributions(g)
            tb = tables.de_tables(qd.p_t_given_x0, qd.output_LLRs, rho, lam, I)
            match = True
        else:
            tb = tables.IBTables(16, 16, g.d_c_max, g.d_v_max, I, arrays["cn"], arrays["vn"], arrays["mc"], arrays["mv"])
        S = a.sub_batch if 0 < a.sub_batch < B else B
        if B % S:
            raise SystemExit("--sub-batch must divide the batch")
        return engine.IBDecoder(G, tb, match, S, path=a.path), match
    kind = 0 if a.kind == "minsum" else 1
    return engine.FloatDecoder(G, kind, I, B, precision=torch.float32, path=a.path), match


def decoder_path(a, dec, B):
    """Which kernels decode a batch of B: {"fused", "small", "folded", "name"} — the fused on-chip kernel,
    the small-batch per-pass kernels (B <= the decoder's small_batch; they do not fold) or the per-pass
    kernels (float: with `folded` degree-2 variables folded into the check pass)."""
    fused = dec.fused
    small = (not fused) and B <= getattr(dec, "small_batch", 0) and (a.kind != "ib" or getattr(dec, "fast_path", False))
    folded = 0 if (a.kind == "ib" or fused or small) else dec.folded
    name = "fused on-chip kernel" if fused else ("small-batch per-pass kernels" if small else "per-pass kernels")
    return {"fused": bool(fused), "small": bool(small), "folded": int(folded), "name": name}


def main():
    a = parse()
    import torch

    from informationbottleneckdecodingldpc_amd import distributed, engine
    from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0

    rank, world, dev = distributed.init_from_env()
    if dev.type != "cuda":
        raise SystemExit("bench.py needs a HIP device")
    B, I = a.batch_per_gpu, a.imax

    # ---- setup: rank 0 builds H + tables, one broadcast to every rank (RCCL over xGMI)
    arrays = distributed.broadcast_arrays(setup_arrays(a) if rank == 0 else None, src=0)
    g = graph_of(arrays)
    n_v = g.n_v
    G = engine.Graph(g, dev)
    q = UniformQuantizer(sigma2_from_ebn0(a.ebn0, g.R_c), 16)
    # channel of global batch gb = batch_offset + rank: the device Philox stream (ibl_channel_sample) under key
    # CH_SEED at counter gb * philox_blocks(N, B) — the frames a 1-GPU run with --batch-offset gb decodes, so a
    # k-GPU line's decoded_bit_errors equals the sum of the 1-GPU lines over the same global batches
    gbatch = a.batch_offset + rank
    ch_offset = gbatch * engine.philox_blocks(n_v, B)
    L = __import__("informationbottleneckdecodingldpc_amd._lib", fromlist=["x"]).load()
    early = bool(a.early_stop)
    its = torch.zeros(max(a.steps, 1), dtype=torch.int32, device=dev)   # stop iteration of every timed step
    step_k = [0]

    def it_slot():
        return its[min(step_k[0], its.numel() - 1):][:1]

    dec, match = build_decoder(a, G, g, arrays, q, B)
    if a.kind == "ib":
        S = dec.max_batch
        ch = torch.empty((n_v, B), dtype=torch.uint8, device=dev)
        engine.channel_sample(ch, q.cdf_t_given_x_equals_zero, CH_SEED, ch_offset)
        out = torch.empty((n_v, B), dtype=torch.uint8, device=dev)
        if S == B:
            run = lambda: dec.decode(ch, out=out, early_stop=early, iters=it_slot())     # noqa: E731
        else:   # contiguous [N][S] pieces, decoded one after another on the stream
            chs = [ch[:, k * S:(k + 1) * S].contiguous() for k in range(B // S)]
            outs = [torch.empty((n_v, S), dtype=torch.uint8, device=dev) for _ in chs]

            def run():
                for c_, o_ in zip(chs, outs):
                    dec.decode(c_, out=o_, early_stop=early, iters=it_slot())
                out.copy_(torch.cat(outs, dim=1))
        timing_on = lambda on: L.ibl_ib_timing(dec._h, int(on))    # noqa: E731
        timing_read_fn = L.ibl_ib_timing_read
        w, dtype = 1, "u8"
    else:
        llr = torch.empty((n_v, B), dtype=torch.float32, device=dev)
        engine.channel_sample(llr, q.cdf_t_given_x_equals_zero, CH_SEED, ch_offset, llr=q.output_LLRs)
        out = torch.empty((n_v, B), dtype=torch.float32, device=dev)
        run = lambda: dec.decode(llr, out=out, early_stop=early, iters=it_slot())    # noqa: E731
        timing_on = lambda on: L.ibl_float_timing(dec._h, int(on))  # noqa: E731
        timing_read_fn = L.ibl_float_timing_read
        w, dtype = 4, "f32"

    import ctypes

    def timing_read():
        cm, vm = ctypes.c_double(), ctypes.c_double()
        cn_, vn_ = ctypes.c_int32(), ctypes.c_int32()
        timing_read_fn(dec._h, ctypes.byref(cm), ctypes.byref(cn_), ctypes.byref(vm), ctypes.byref(vn_))
        return cm.value, cn_.value, vm.value, vn_.value

    for _ in range(a.warmup):
        run()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(a.steps):
        step_k[0] = k
        if k == a.steps - 1 and not a.no_kernel_events:
            timing_on(True)      # HIP events around the launches of the last timed step only
        run()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    elapsed_local = time.perf_counter() - t0
    timing_on(False)
    cn_ms, cn_n, vn_ms, vn_n = timing_read()

    # errors of the decoded batch (sanity: counted on device, outside the timed region)
    errs = int(engine.count_below(out, g.data_len, 8 if a.kind == "ib" else 0.0).item())
    tot = distributed.allreduce_counts({"errors": errs, "bits": g.data_len * B})

    agg = aggregate_rate(B, a.steps, elapsed_local)
    elapsed, value = agg["elapsed_max_s"], agg["value"]
    bpc = bytes_per_cw(g.n_e, n_v, I, w)
    cn_avg, vn_avg = cn_ms / max(cn_n, 1), vn_ms / max(vn_n, 1)
    kpath = decoder_path(a, dec, B)
    fused, small, folded = kpath["fused"], kpath["small"], kpath["folded"]
    stop_it = its[:a.steps].cpu().numpy() if a.steps > 0 else np.zeros(1, np.int32)
    fast = a.kind == "ib" and getattr(dec, "fast_path", False)
    # bytes per stored message / channel value as this build moves them: the IB fast path keeps 4-bit
    # nibbles (2 codewords per byte), the generic IB path u8, the float paths fp32
    ws = 0.5 if fast else w
    fmt = "u4" if fast else ("u8" if a.kind == "ib" else "f32")
    if a.kind == "ib":
        dtype = fmt
    roof = roofline(a, g, n_v, B, I, w, ws, fmt, match, fused, cn_avg, vn_avg, cn_ms, vn_ms, cn_n, vn_n, dec,
                    folded=folded, small=small)
    # HBM bytes the decode moves per codeword at the stored widths (channel in, output out: u8 for IB, fp32 float)
    moved = moved_bytes_per_cw(g.n_e, n_v, I, "fused" if fused else "passes", ws, w, w, w_stage=w, folded=folded)
    cpu = None
    code_name, code_desc = CODES[a.code]
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not early:   # the baseline times fixed iterations
        cpu = cpu_baseline(a, g, arrays, I, B, match, ch if a.kind == "ib" else llr, out, code_name)

    if rank == 0:
        line = {
            "metric": ("decoded codewords/sec + achieved HBM GB/s, DVB-S2 N=64800 i_max=50"
                       if (a.code, a.kind, I) == ("dvbs2", "ib", 50) else
                       f"decoded codewords/sec + achieved HBM GB/s, {code_name} {a.kind} i_max={I}"),
            "value": round(value, 1),
            "unit": "codewords/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": f"synthetic: all-zero codeword, BPSK/AWGN at Eb/N0 {a.ebn0} dB quantised to 16 clusters "
                    f"(device Philox, key {CH_SEED}, global batch {a.batch_offset}+rank); "
                    f"{('DE-designed T=16 IB tables (0.75 dB)' if early else 'random T=16 IB tables') if a.kind == 'ib' else 'cluster LLRs'}"
                    f"; {code_desc}",
            "config": {"workload": f"{code_name}, "
                                   f"{'IB-LUT T=16' if a.kind == 'ib' else a.kind + ' fp32'}, i_max={I}, "
                                   f"{B} codewords per GPU, "
                                   f"{('matching ' + ('on' if match else 'off') + ', ') if a.kind == 'ib' else ''}"
                                   f"{kpath['name']}"
                                   f"{', early stop on (batch-global)' if early else ', fixed iterations'}",
                       "batch_per_gpu": B, "global_batch": B * world, "imax": I, "parallelism": f"dp{world} batch split",
                       "early_stop": early, "ebn0_db": a.ebn0, "batch_offset": a.batch_offset,
                       "sub_batch": a.sub_batch or None,
                       "baseline_config": a.config or ("C4" if (a.code, a.kind, I) == ("dvbs2", "ib", 50) else None)},
            "hbm_gbps_algorithmic": round(value * moved / 1e9, 1),
            "bytes_per_codeword": int(round(moved)),
            "hbm_gbps_u8_equivalent": round(value * bpc / 1e9, 1),
            "bytes_per_codeword_u8_equivalent": bpc,
            "hbm_note": ("hbm_gbps_algorithmic = codewords/s x the bytes the kernels move per codeword at their stored "
                         f"widths ({fmt} messages{', fused on-chip: channel in + output out only' if fused else ''}); "
                         "*_u8_equivalent = SURVEY §8(d)'s fixed 1-byte reporting width, not bytes moved"),
            "dist": {k: (round(v, 6) if isinstance(v, float) else
                         ({a_: round(b_, 1) for a_, b_ in v.items()} if isinstance(v, dict) else v))
                     for k, v in agg.items() if k != "value"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "decoded_bit_errors": tot["errors"], "decoded_bits": tot["bits"],
            # stop iteration L the decoder reports (ibl_*_decode d_iters; i_max - 1 = ran every iteration), rank 0
            "stop_iteration": {"min": int(stop_it.min()), "max": int(stop_it.max()), "imax": I},
            "latency_ms_per_decode": round(elapsed / max(a.steps, 1) * 1e3, 4),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
