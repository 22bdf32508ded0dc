#!/bin/bash
# Round-6 GPU session i: small-batch decodes, eager launches vs one graph replay per decode.
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
for k in ib bp; do
  for b in 2 32; do
    timeout -k 10 200 python tools/graph_small.py --kind $k --batch $b --reps $([ $k = ib ] && echo 300 || echo 60) > $O/graph_${k}_b$b.json 2> $O/graph_${k}_b$b.err || exit 1
  done
done
