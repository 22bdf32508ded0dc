"""Diagnostic (GPU box): fp32 GPU decoders vs the CPU oracles, per i_max.

  * min-sum fp32 GPU vs the fp32 oracle (bit-exact expected) and vs the fp64 oracle (divergence);
  * BP fp32 GPU vs the fp64 oracle (max relative error, share outside SURVEY H5's
    1e-5*max(|x|,|y|) + 1e-4, hard-decision flips).

usage: python tools/diag_float32.py [minsum|bp|all] [B]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from informationbottleneckdecodingldpc_amd import codes, engine, graph  # noqa: E402
from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0  # noqa: E402
from oracle import oracle  # noqa: E402


def stats(out, ref):
    err = np.abs(out - ref)
    mx = np.maximum(np.abs(out), np.abs(ref))
    rel = err / np.maximum(mx, 1e-30)
    h5 = err > 1e-5 * mx + 1e-4
    return (f"max_abs={err.max():.2e} max_rel={rel.max():.2e} out_of_H5={h5.mean():.2e} "
            f"hard_flips={int(((out < 0) != (ref < 0)).sum())}/{out.size}")


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    if what in ("minsum", "all"):
        g = graph.build_graph(codes.wlan_80211n(81))
        G = engine.Graph(g, "cuda:0")
        for ebn0 in (1.0, 2.0, 3.0):
            q = UniformQuantizer(sigma2_from_ebn0(ebn0, g.R_c), 16)
            llr = q.llr_of(q.sample_all_zero(g.n_v, 256, np.random.default_rng(1))).astype(np.float32)
            for imax in (2, 5, 10, 20, 30, 50):
                r32 = oracle.float32_decode(g, imax, llr).astype(np.float64)
                r64 = oracle.float_decode(g, 0, imax, llr.astype(np.float64))
                d = engine.FloatDecoder(G, 0, imax, llr.shape[1], precision=torch.float32)
                out = d.decode(torch.from_numpy(llr).cuda(), early_stop=False).double().cpu().numpy()
                print(f"minsum wlan1944 {ebn0} dB imax={imax}: gpu==fp32 oracle {np.array_equal(out, r32)}; "
                      f"fp32 vs fp64: {stats(out, r64)}", flush=True)
    if what in ("bp", "all"):
        for name, H, imaxs in (("dvbs2", codes.dvbs2_structured(seed=0), (2, 5, 10, 20, 50, 100)),
                               ("wlan1944", codes.wlan_80211n(81), (2, 5, 10, 20, 50, 100))):
            g = graph.build_graph(H)
            G = engine.Graph(g, "cuda:0")
            for ebn0 in (0.6, 1.0, 1.5, 2.0):
                q = UniformQuantizer(sigma2_from_ebn0(ebn0, g.R_c), 16)
                llr = q.llr_of(q.sample_all_zero(g.n_v, B, np.random.default_rng(2)))
                for imax in imaxs:
                    r64, it64 = oracle.float_decode(g, 1, imax, llr, early_stop=True, return_iters=True)
                    d = engine.FloatDecoder(G, 1, imax, B, precision=torch.float32)
                    it = torch.zeros(1, dtype=torch.int32, device="cuda:0")
                    out = d.decode(torch.from_numpy(llr).cuda().float(), early_stop=True, iters=it)
                    out = out.double().cpu().numpy()
                    print(f"bp {name} {ebn0} dB imax={imax}: stop {int(it.item())} vs {it64}; {stats(out, r64)}",
                          flush=True)


if __name__ == "__main__":
    main()
