#!/bin/bash
# Round-6 final session t: full GPU suite, smoke, every config's bench line, BER driver (two slice sizes).
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
CONFIGS="C4 C1 C2 C3 C5" bash tools/gpu_run.sh r6t tests smoke bench || exit 1
timeout -k 10 400 python tools/bench_ber.py --cases c4,c4enc,c5 --batches 16 --gen-chunk 4194304,0 > $O/bench_ber.json 2> $O/bench_ber.err || exit 1
