#!/bin/bash
# Round-6 GPU session q: does the kernarg placement matter for the B=2 launch chain? (HIP_FORCE_DEV_KERNARG)
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
for v in unset 1 0; do
  if [ $v = unset ]; then
    timeout -k 10 200 python tools/graph_small.py --kind ib --batch 2 --reps 300 > $O/ib_$v.json 2> $O/ib_$v.err || exit 1
  else
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python tools/graph_small.py --kind ib --batch 2 --reps 300 > $O/ib_$v.json 2> $O/ib_$v.err || exit 1
  fi
done
env | grep -i "^HIP_\|^HSA_\|^GPU_" > $O/env.txt || true
