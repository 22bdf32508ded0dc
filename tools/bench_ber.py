"""End-to-end BER-driver throughput on one GPU: `ber.run_ber` over the reference-named drop-in
classes, as `DVB-S2/BER_simulation_OpenCL.py:95-121` drives them — per batch the device channel
(`quantize_direct_OpenCL[_LLR]`), the decode (`decode_OpenCL[_belief_propagation]`, early stop on), the error
count (`return_errors_all_zero`) and the host-side stop rule. One Eb/N0 point, a fixed number of batches
(`max_blocks`), timed by the driver itself (`BERResult.seconds`: the point's loop, after the decoder is built).
`value` is the pipelined driver (round 6: channel of batch k+1 on a side stream while batch k decodes, counts
on the side stream, one host read per round); `sync_driver` the reference call sequence batch by batch; and
`decode_only` the same decoder decoding a resident channel back to back, measured in the same process.

  python tools/bench_ber.py [--batches K] [--cases c4,c4enc,c5] [--gen-chunk 4194304,0]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(case, batches, B, gen_chunk=None):
    import torch
    from informationbottleneckdecodingldpc_amd import codes, engine, graph, tables
    from informationbottleneckdecodingldpc_amd.ber import BERConfig, run_ber
    from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0
    H = codes.dvbs2_structured(seed=0)
    g = graph.build_graph(H)
    ebn0 = 1.0
    # sync_every divides the batch count: run_ber decodes whole rounds of sync_every batches and discards the
    # ones past the stop, which would otherwise be decoded inside the timed loop but not counted
    sync = max(k for k in (4, 2, 1) if batches % k == 0)
    cfg = dict(EbN0_dB_start=ebn0, EbN0_dB_max_value=ebn0, target_error_rate=1.0, min_errors=10 ** 12,
               msg_at_time=B, max_blocks=batches * B, sync_every=sync, seed=2)
    if case.startswith("c4"):
        from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import \
            Discrete_LDPC_Decoder_class_irregular
        q = UniformQuantizer(sigma2_from_ebn0(0.75, g.R_c), 16)      # DE tables designed at 0.75 dB (round 6)
        rho, lam = tables.edge_degree_distributions(g)
        tb = tables.de_tables(q.p_t_given_x0, q.output_LLRs, rho, lam, 50)
        dec = Discrete_LDPC_Decoder_class_irregular(H, 50, 16, 16, tb.cn, tb.vn, tb.match_cn, tb.match_vn, B,
                                                    match="true")
        cfg["encoded"] = case == "c4enc"
        what = "IB T=16 i_max=50 (DE tables designed at 0.75 dB), Discrete_LDPC_Decoder_class_irregular"
    else:
        from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular
        dec = BeliefPropagationDecoderClassIrregular(H, 100, 16, B)
        cfg["llr_dtype"] = torch.float32
        what = "BP fp32 i_max=100, BeliefPropagationDecoderClassIrregular"
    if gen_chunk is not None:
        cfg["gen_chunk"] = gen_chunk
    run_ber(dec, BERConfig(**{**cfg, "max_blocks": B}))          # warm-up: decoder, streams, allocator
    r = run_ber(dec, BERConfig(**cfg))
    rs = run_ber(dec, BERConfig(**cfg, pipeline=False))          # the reference call sequence, batch by batch
    assert r.errors == rs.errors and r.blocks == rs.blocks
    sec, sec_s = r.seconds[0], rs.seconds[0]
    # decode-only on the same decoder object, batch and early-stop setting: the drop-in decode of a channel
    # already resident in HBM, back to back (what bench.py's line measures), same number of batches
    # With early stop on, a batch's decode time depends on its frames: where the driver's batches fit in 1 GiB the
    # decode-only line decodes as many fresh channels (consecutive Philox batches), else one resident channel again.
    nb = r.blocks[0] // B
    dt = torch.uint8 if case.startswith("c4") else torch.float32
    q = UniformQuantizer(sigma2_from_ebn0(ebn0, g.R_c), 16)
    fresh = nb * g.n_v * B * (1 if case.startswith("c4") else 4) <= 1 << 30
    xs = []
    for k in range(nb if fresh else 1):
        x = torch.empty((g.n_v, B), dtype=dt, device="cuda")
        engine.channel_sample(x, q.cdf_t_given_x_equals_zero, 2, k * engine.philox_blocks(g.n_v, B),
                              llr=None if case.startswith("c4") else q.output_LLRs)
        xs.append(x)
    # (IB: u8 decisions, as the pipelined driver asks for them — the same cluster ids as the reference's int32)
    kw = {"out_dtype": torch.uint8} if case.startswith("c4") else {}
    fn = dec.decode_OpenCL if case.startswith("c4") else dec.decode_OpenCL_belief_propagation
    fn(xs[0], buffer_in=True, return_buffer=True, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(nb):
        fn(xs[k % len(xs)], buffer_in=True, return_buffer=True, **kw)
    torch.cuda.synchronize()
    dec_only = r.blocks[0] / (time.perf_counter() - t0)
    value = r.blocks[0] / sec
    return {"metric": "BER-driver decoded codewords/sec (run_ber: channel + decode + error count + stop rule)",
            "case": case, "code": "DVB-S2-structured N=64800 R=1/2", "decoder": what,
            "encoded_codewords": bool(cfg.get("encoded")), "ebn0_db": ebn0, "batch": B, "batches": r.blocks[0] // B,
            "sync_every": sync, "early_stop": True, "value": round(value, 1), "unit": "codewords/s",
            "seconds": round(sec, 4), "sync_driver": {"value": round(r.blocks[0] / sec_s, 1), "seconds": round(sec_s, 4),
                                                      "note": "cfg.pipeline=False: quantise -> decode -> count per batch"},
            "decode_only": {"value": round(dec_only, 1), "fresh_channels": fresh,
                            "note": "the same drop-in decode on resident channels, back to back, same batch count "
                                    "(fresh_channels: one per batch, else one channel decoded again)"},
            "vs_decode_only": round(value / dec_only, 4), "gen_chunk": BERConfig(**cfg).gen_chunk,
            "errors": r.errors[0], "errors_equal_sync_driver": True, "ber": float(r.BER_vector[0])}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batches", type=int, default=8)
    p.add_argument("--batch", type=int, default=8192)
    p.add_argument("--cases", default="c4,c4enc,c5")
    p.add_argument("--gen-chunk", default=None, help="comma list of BERConfig.gen_chunk values to A/B (0 = one launch a batch)")
    a = p.parse_args()
    chunks = [None] if a.gen_chunk is None else [int(x) for x in a.gen_chunk.split(",")]
    for c in a.cases.split(","):
        for gc in chunks:
            print(json.dumps(run(c, a.batches if c != "c5" else max(2, a.batches // 2), a.batch, gc)), flush=True)


if __name__ == "__main__":
    main()
