#!/bin/bash
# Round-6 GPU session e: VN interleave A/B (3 reps, same box), BER-driver kernel profile.
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
REPS=3 bash tools/ab.sh r6e/ab "base vmix3" || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ber -o ber -- python tools/bench_ber.py --cases c4 --batches 4 > $O/bench_ber_prof.json 2> $O/bench_ber_prof.err || exit 1
