#!/bin/bash
# Round-6 GPU session j: BP B=2 in bench.py vs tools/graph_small.py on one box, kernel traces of both.
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 200 python bench.py --config C5 --batch-per-gpu 2 --steps 50 --warmup 5 --no-cpu-baseline --no-kernel-events > $O/bench_bp_b2.json 2> $O/bench_bp_b2.err || exit 1
timeout -k 10 200 python tools/graph_small.py --kind bp --batch 2 --reps 60 > $O/graph_bp_b2.json 2> $O/graph_bp_b2.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_bench -o run -- python3 bench.py --config C5 --batch-per-gpu 2 --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-events > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_tool -o run -- python3 tools/graph_small.py --kind bp --batch 2 --reps 10 > $O/trace_tool.json 2> $O/trace_tool.err || exit 1
