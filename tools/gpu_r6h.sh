#!/bin/bash
# Round-6 GPU session h: small-batch thresholds and launch gaps after packing the small-batch rows.
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
LINES=tools/lines_thresh.txt bash tools/gpu_run.sh r6h lines || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_b2 -o run -- python3 bench.py --config C4 --batch-per-gpu 2 --steps 20 --warmup 2 --no-cpu-baseline --no-kernel-events > $O/trace_b2.json 2> $O/trace_b2.err || exit 1
