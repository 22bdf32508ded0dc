#!/bin/bash
# Round-6 GPU session d: counters / channel tests, BER-driver throughput, DVB-S2 BER curves, rank rehearsals.
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_channel.py tests/test_gpu_encoder.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_channel.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_ber.py --cases c4,c4enc,c5 > $O/bench_ber.json 2> $O/bench_ber.err || exit 1
timeout -k 10 600 python tools/ber_curves.py > $O/ber_curves.json 2> $O/ber_curves.err || exit 1
timeout -k 10 300 python tools/sweep_ranks.py > $O/sweep_w1.json 2> $O/sweep_w1.err || exit 1
IBL_SHARE_DEVICE=1 IBL_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 tools/sweep_ranks.py > $O/sweep_w2.json 2> $O/sweep_w2.err || exit 1
IBL_SHARE_DEVICE=1 IBL_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 8 --steps 2 --warmup 1 > $O/mrank8_C4.json 2> $O/mrank8_C4.err || exit 1
for o in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 python bench.py --batch-offset $o --steps 1 --warmup 0 --no-cpu-baseline >> $O/rank1_offsets_C4.jsonl 2>> $O/rank1_offsets.err || exit 1
done
