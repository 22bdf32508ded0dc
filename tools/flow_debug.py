"""One fused float decode (WLAN N=1296 min-sum fp32, B=301, i_max=10) with the task dataflow, then its
health words (ibl_float_flow_status) and parity against the barrier schedule: python tools/flow_debug.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from informationbottleneckdecodingldpc_amd import codes, engine, graph  # noqa: E402
from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0  # noqa: E402

g = graph.build_graph(codes.wlan_80211n())
B, imax = int(sys.argv[1]) if len(sys.argv) > 1 else 301, 10
q = UniformQuantizer(sigma2_from_ebn0(1.5, g.R_c), 16)
llr = q.llr_of(q.sample_all_zero(g.n_v, B, np.random.default_rng(1))).astype(np.float32)
G = engine.Graph(g, "cuda:0")
outs = {}
for flow in ("1", "0"):
    os.environ["IBL_FUSED_FLOW"] = flow
    dec = engine.FloatDecoder(G, 0, imax, B, precision=torch.float32, path="fused")
    out = dec.decode(torch.from_numpy(llr).cuda(), early_stop=False)
    torch.cuda.synchronize()
    st = dec.flow_status()
    print(f"flow={flow} in_use={dec.flow} status={st[:8]}", flush=True)
    if st[0]:
        print(" stamps c:", st[8:8 + 64], "\n stamps v:", st[72:136], flush=True)
    outs[flow] = out.cpu().numpy()
print("equal:", bool(np.array_equal(outs["1"], outs["0"])), flush=True)
