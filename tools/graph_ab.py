"""A/B: the C4 decode issued directly vs replayed from a captured HIP graph (torch.cuda.CUDAGraph over the
C ABI's launches on the capturing stream). Prints one JSON line per mode."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from informationbottleneckdecodingldpc_amd import codes, engine, graph, tables  # noqa: E402
from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0  # noqa: E402

B, I, STEPS = 8192, 50, int(os.environ.get("STEPS", "10"))
dev = torch.device("cuda:0")
g = graph.build_graph(codes.dvbs2_structured(seed=0))
tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, I, seed=1)
dec = engine.IBDecoder(engine.Graph(g, dev), tb, True, B)
q = UniformQuantizer(sigma2_from_ebn0(0.6, g.R_c), 16)
gen = torch.Generator(device=dev)
gen.manual_seed(3)
ch = q.sample_all_zero_device(g.n_v, B, dev, generator=gen)
out = torch.empty((g.n_v, B), dtype=torch.uint8, device=dev)
s = torch.cuda.Stream(dev)
with torch.cuda.stream(s):
    for _ in range(2):
        dec.decode(ch, out=out, early_stop=False)
torch.cuda.synchronize()
ref = out.clone()


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / STEPS


with torch.cuda.stream(s):
    direct = timed(lambda: dec.decode(ch, out=out, early_stop=False))
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr, stream=s):
    dec.decode(ch, out=out, early_stop=False)
out.zero_()
gr.replay()
torch.cuda.synchronize()
same = bool(torch.equal(out, ref))
graphed = timed(gr.replay)
for mode, t in (("direct", direct), ("graph", graphed)):
    print(json.dumps({"mode": mode, "ms_per_step": round(t * 1e3, 3), "codewords_per_s": round(B / t, 1),
                      "graph_output_equal": same}))
