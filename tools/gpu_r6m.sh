#!/bin/bash
# Round-6 GPU session m: counters of the B=2 small-batch kernels (IB vs BP), one pass per counter set.
set -o pipefail
O=gpurun_out/r6m
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for k in ib bp; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d $R/$O/sq_$k -o run --output-format csv -- python3 $R/tools/graph_small.py --kind $k --batch 2 --reps 3 > $R/$O/sq_$k.json 2> $R/$O/sq_$k.err || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum -d $R/$O/tcc_$k -o run --output-format csv -- python3 $R/tools/graph_small.py --kind $k --batch 2 --reps 3 > $R/$O/tcc_$k.json 2> $R/$O/tcc_$k.err || exit 1
done
