#!/bin/bash
# Round-6 GPU session r: binned CDF inversion in the channel sampler: parity, BER-driver throughput, kernel stats.
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_channel.py tests/test_gpu_encoder.py tests/test_gpu_ber_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_ber.py --cases c4,c4enc,c5 > $O/bench_ber.json 2> $O/bench_ber.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ber -o ber --output-format csv -- python tools/bench_ber.py --cases c4 --batches 4 > $O/bench_ber_prof.json 2> $O/bench_ber_prof.err || exit 1
