#!/bin/bash
# Round-6 GPU session f: parity of the rewritten staging / counters / channel slices, BER-driver throughput, C4 bench.
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ib.py tests/test_gpu_channel.py tests/test_gpu_encoder.py tests/test_gpu_ber_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_ber.py --cases c4,c4enc,c5 > $O/bench_ber.json 2> $O/bench_ber.err || exit 1
timeout -k 10 200 python bench.py > $O/bench_C4.json 2> $O/bench_C4.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ber -o ber --output-format csv -- python tools/bench_ber.py --cases c4 --batches 4 > $O/bench_ber_prof.json 2> $O/bench_ber_prof.err || exit 1
