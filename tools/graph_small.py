"""Small-batch decodes: eager launches vs one hipGraph replay per decode (diagnostic).

At B = 2 a DVB-S2 decode is ~100 dependent launches of a few microseconds each; this measures what the launch
chain costs by capturing one whole decode (torch.cuda.CUDAGraph around the drop-in decode call, which launches
on the current stream) and replaying it, against the same decode launched eagerly, and checks that both give
the same decisions.

  python tools/graph_small.py [--kind ib|bp] [--batch 2] [--reps 200]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kind", choices=["ib", "bp"], default="ib")
    p.add_argument("--batch", type=int, default=2)
    p.add_argument("--reps", type=int, default=200)
    a = p.parse_args()
    import torch

    import bench
    from informationbottleneckdecodingldpc_amd import engine
    from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0
    ba = bench.parse(["--config", "C4" if a.kind == "ib" else "C5", "--batch-per-gpu", str(a.batch)])
    dev = torch.device("cuda:0")
    arrays = bench.setup_arrays(ba)
    g = bench.graph_of(arrays)
    G = engine.Graph(g, dev)
    q = UniformQuantizer(sigma2_from_ebn0(ba.ebn0, g.R_c), 16)
    B = a.batch
    dec, _ = bench.build_decoder(ba, G, g, arrays, q, B)
    if a.kind == "ib":
        x = torch.empty((g.n_v, B), dtype=torch.uint8, device=dev)
        engine.channel_sample(x, q.cdf_t_given_x_equals_zero, bench.CH_SEED, 0)
        out = torch.empty((g.n_v, B), dtype=torch.uint8, device=dev)
    else:
        x = torch.empty((g.n_v, B), dtype=torch.float32, device=dev)
        engine.channel_sample(x, q.cdf_t_given_x_equals_zero, bench.CH_SEED, 0, llr=q.output_LLRs)
        out = torch.empty((g.n_v, B), dtype=torch.float32, device=dev)
    s = torch.cuda.Stream(dev)
    res = {"kind": a.kind, "batch": B, "reps": a.reps, "imax": ba.imax}
    with torch.cuda.stream(s):
        for _ in range(5):
            dec.decode(x, out=out, early_stop=False)
        torch.cuda.synchronize(dev)
        ref = out.clone()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            dec.decode(x, out=out, early_stop=False)
        torch.cuda.synchronize(dev)
        res["eager_ms_per_decode"] = (time.perf_counter() - t0) * 1e3 / a.reps
        out.zero_()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            dec.decode(x, out=out, early_stop=False)
        for _ in range(5):
            gr.replay()
        torch.cuda.synchronize(dev)
        res["graph_equal"] = bool(torch.equal(out, ref))
        t0 = time.perf_counter()
        for _ in range(a.reps):
            gr.replay()
        torch.cuda.synchronize(dev)
        res["graph_ms_per_decode"] = (time.perf_counter() - t0) * 1e3 / a.reps
    res["eager_cw_per_s"] = B / res["eager_ms_per_decode"] * 1e3
    res["graph_cw_per_s"] = B / res["graph_ms_per_decode"] * 1e3
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
