#!/bin/bash
# Round-6 GPU session l: kernel traces of IB and BP B=2 decodes on one box.
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in ib bp; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$k -o run -- python3 tools/graph_small.py --kind $k --batch 2 --reps 20 > $O/trace_$k.json 2> $O/trace_$k.err || exit 1
done
