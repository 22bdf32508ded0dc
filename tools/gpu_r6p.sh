#!/bin/bash
# Round-6 GPU session p: thresholds without kernel events; BP B=2 kernel trace after the grid-size fix.
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
LINES=tools/lines_thresh2.txt bash tools/gpu_run.sh r6p lines || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_bp -o run -- python3 tools/graph_small.py --kind bp --batch 2 --reps 20 > $O/trace_bp.json 2> $O/trace_bp.err || exit 1
