"""DVB-S2 BER curves of the IB decoder with density-evolution tables against BP on the same frames.

Every decoder runs through the BER driver (`ber.run_ber`, the reference's DVB-S2 driver loop over the drop-in classes)
with the same seed, batch and block count per point, so each point decodes the identical channel frames (the device
Philox stream keyed on the global batch index; IB gets the clusters, BP their fp32 LLRs):

  * IB T=16, i_max=50, matching, tables from `tables.de_tables` designed at one Eb/N0 per curve (`--designs`,
    default 0.75 and 0.8 dB: the reference's DVB-S2 configs are designed at one point too,
    DVB-S2/decoder_config_generation.py:20);
  * IB T=16 with the round-5 fixed-alphabet `llr_tables` (designed per point) for comparison;
  * BP fp32 (BeliefPropagationDecoderClassIrregular) at i_max 50 and 100.

  python tools/ber_curves.py [--points 0.8:1.3:0.05] [--batches 4] [--batch 8192] > profiles/r06_dvbs2_ber_curves.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--points", default="0.8:1.3:0.05")
    p.add_argument("--batches", type=int, default=4)
    p.add_argument("--batch", type=int, default=8192)
    p.add_argument("--designs", default="0.75,0.8", help="design Eb/N0 of the DE tables, one IB curve each")
    p.add_argument("--decoders", default="ib_de,ib_llr,bp50,bp100")
    a = p.parse_args()
    import torch
    from informationbottleneckdecodingldpc_amd import codes, graph, tables
    from informationbottleneckdecodingldpc_amd.ber import BERConfig, run_ber
    from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular
    from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0
    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import Discrete_LDPC_Decoder_class_irregular
    lo, hi, st = (float(x) for x in a.points.split(":"))
    pts = [round(x, 4) for x in np.arange(lo, hi + st / 2, st)]
    H = codes.dvbs2_structured(seed=0)
    g = graph.build_graph(H)
    rho, lam = tables.edge_degree_distributions(g)
    B = a.batch
    t0 = time.time()
    designs = [float(x) for x in a.designs.split(",")]
    des = {}
    for dz in designs:
        qd = UniformQuantizer(sigma2_from_ebn0(dz, g.R_c), 16)
        des[f"ib_de{dz:g}"] = tables.de_tables(qd.p_t_given_x0, qd.output_LLRs, rho, lam, 50)
    design_s = (time.time() - t0) / len(designs)
    names = []
    for n in a.decoders.split(","):
        names += list(des) if n == "ib_de" else [n]
    curves = {}
    for name in names:
        ber, errs, secs = [], [], []
        for x in pts:
            if name in des:
                tb = des[name]
            elif name == "ib_llr":
                q = UniformQuantizer(sigma2_from_ebn0(x, g.R_c), 16)
                tb = tables.llr_tables(q.output_LLRs, g.d_c_max, g.d_v_max, 50)
            if name.startswith("ib"):
                dec = Discrete_LDPC_Decoder_class_irregular(H, 50, 16, 16, tb.cn, tb.vn, tb.match_cn, tb.match_vn, B,
                                                            match="true")
                kw = {}
            else:
                dec = BeliefPropagationDecoderClassIrregular(H, int(name[2:]), 16, B, precision=torch.float32)
                kw = {"llr_dtype": torch.float32}
            cfg = BERConfig(EbN0_dB_start=x, EbN0_dB_max_value=x, target_error_rate=1.0, min_errors=10 ** 15,
                            msg_at_time=B, max_blocks=a.batches * B, sync_every=a.batches, seed=7, **kw)
            r = run_ber(dec, cfg)
            ber.append(float(r.BER_vector[0]))
            errs.append(int(r.errors[0]))
            secs.append(round(r.seconds[0], 3))
            del dec
            print(json.dumps({"decoder": name, "ebn0_db": x, "ber": ber[-1], "errors": errs[-1],
                              "blocks": r.blocks[0], "seconds": secs[-1]}), file=sys.stderr, flush=True)
        curves[name] = {"ber": ber, "errors": errs, "seconds": secs}

    def first_below(name, thr):
        for x, b in zip(pts, curves[name]["ber"]):
            if b <= thr:
                return x
        return None
    summary = {k: {"ebn0_ber_le_1e-3": first_below(k, 1e-3), "ebn0_ber_le_1e-4": first_below(k, 1e-4)} for k in curves}
    print(json.dumps({"metric": "DVB-S2 BER curves on identical frames (run_ber, device channel)",
                      "code": "DVB-S2-structured N=64800 R=1/2 (EN 302 307 profile, synthetic addresses)",
                      "channel": "BPSK/AWGN, 16-cluster uniform quantiser (AD_max_abs 3), all-zero codeword, Philox seed 7",
                      "batch": B, "blocks_per_point": a.batches * B, "bits_per_point": a.batches * B * int(g.data_len),
                      "early_stop": "batch-global (never triggers at this batch: the degree-1 parity variable)",
                      "ib_design_ebn0_db": designs, "de_design_seconds_each": round(design_s, 2),
                      "ebn0_db": pts, "curves": curves, "summary": summary}), flush=True)


if __name__ == "__main__":
    main()
