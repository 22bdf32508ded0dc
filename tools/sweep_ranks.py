"""C5's BP sweep through run_ber as k ranks under torchrun: rank r decodes global batches
base + j*k + r, the per-round counts are all-reduced (gloo here: the ranks share one GPU, IBL_SHARE_DEVICE=1) and
every rank walks them in global order, so the sweep must equal the 1-rank sweep point for point.

  python tools/sweep_ranks.py                        # 1 rank
  IBL_SHARE_DEVICE=1 IBL_DIST_BACKEND=gloo torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/sweep_ranks.py
Rank 0 prints one JSON line: world size, backend, points, errors, blocks, BER."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from informationbottleneckdecodingldpc_amd import codes, distributed
    from informationbottleneckdecodingldpc_amd.ber import BERConfig, run_ber
    from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular
    rank, world, dev = distributed.init_from_env()
    H = codes.dvbs2_structured(seed=0)
    B = int(os.environ.get("SWEEP_B", "8"))
    bp = BeliefPropagationDecoderClassIrregular(H, 100, 16, B, precision=torch.float32)
    cfg = BERConfig(EbN0_dB_start=0.2, EbN0_dB_max_value=1.2, EbN0_dB_normal_stepwidth=0.25,
                    EbN0_dB_small_stepwidth=0.125, target_error_rate=1e-9, min_errors=40000, msg_at_time=B,
                    max_blocks=12 * B, seed=31, llr_dtype=torch.float32, sync_every=2)
    r = run_ber(bp, cfg)
    if rank == 0:
        import torch.distributed as dist
        print(json.dumps({"world": world, "backend": dist.get_backend() if dist.is_initialized() else "none",
                          "batch_per_rank": B, "sync_every": cfg.sync_every, "ebn0_db": [float(x) for x in r.EbN0_dB_vector],
                          "errors": [int(e) for e in r.errors], "blocks": list(r.blocks),
                          "ber": [float(x) for x in r.BER_vector], "seconds": [round(s, 3) for s in r.seconds]}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
