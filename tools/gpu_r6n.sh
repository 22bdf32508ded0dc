#!/bin/bash
# Round-6 GPU session n: address-translation and L2-request latency counters of the B=2 kernels (IB vs BP).
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for k in ib bp; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum -d $R/$O/tcp_$k -o run --output-format csv -- python3 $R/tools/graph_small.py --kind $k --batch 2 --reps 3 > $R/$O/tcp_$k.json 2> $R/$O/tcp_$k.err || exit 1
done
