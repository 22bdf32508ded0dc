"""Encoder throughput on one GPU (SURVEY §8(f) "next" #4, DESIGN.md "Encoder"): batched systematic encoding
of random information words through `engine.Encoder` (the C-ABI `ibl_encode`), inputs resident in HBM,
timed with HIP events on the encoder's stream. One JSON line per code.

  python tools/bench_encoder.py [--steps K] [--warmup W] [--codes dvbs2,wlan1944]

`bytes_per_codeword` = K information bytes read + N codeword bytes written at the API's u8 [rows][B] layout
(the interface traffic; the kernels' internal bit-packed words are extra)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from informationbottleneckdecodingldpc_amd import codes, engine  # noqa: E402

CODES = {"dvbs2": (lambda: codes.dvbs2_structured(seed=0), 8192), "wlan1944": (lambda: codes.wlan_80211n(81), 65536)}


def run(name, steps, warmup):
    make, B = CODES[name]
    H = make()
    dev = torch.device("cuda", 0)
    enc = engine.Encoder(H, B, dev)
    info = torch.empty((enc.K, B), dtype=torch.uint8, device=dev)
    engine.random_bits(info, seed=7, offset=0)
    out = torch.empty((enc.N, B), dtype=torch.uint8, device=dev)
    for _ in range(warmup):
        enc.encode(info, out)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(steps):
        enc.encode(info, out)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    # every codeword satisfies H x = 0 (checked on the last step's output)
    Hc = H.tocoo()
    Hd = torch.sparse_coo_tensor(torch.from_numpy(np.stack([Hc.row, Hc.col]).astype(np.int64)), torch.ones(Hc.nnz),
                                 Hc.shape).to(dev)
    syn = torch.remainder(torch.sparse.mm(Hd, out[:, :64].float()), 2).abs().sum().item()
    bpc = enc.K + enc.N
    return {"metric": "encoded codewords/sec", "code": name, "N": enc.N, "K": enc.K, "batch": B,
            "algorithm": enc.algorithm, "ms_per_batch": round(ms, 4), "value": round(B / (ms * 1e-3), 1),
            "unit": "codewords/s", "bytes_per_codeword": bpc, "gbps_interface": round(B * bpc / (ms * 1e-3) / 1e9, 1),
            "syndrome_weight_first64": syn, "steps": steps, "warmup": warmup}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--codes", default="dvbs2,wlan1944")
    a = p.parse_args()
    for name in a.codes.split(","):
        print(json.dumps(run(name, a.steps, a.warmup)), flush=True)


if __name__ == "__main__":
    main()
