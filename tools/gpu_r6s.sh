#!/bin/bash
# Round-6 GPU session s: binned channel inversion (kernarg table) vs T compares (variant chloop): parity, BER driver
# A/B over two repetitions, with the side-stream slices (4M samples) and one launch per batch (gen_chunk 0).
set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
V=informationbottleneckdecodingldpc_amd/variants
timeout -k 10 500 python -u -m pytest tests/test_gpu_ib.py tests/test_gpu_channel.py tests/test_gpu_ber_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 400 python tools/bench_ber.py --cases c4 --batches 16 --gen-chunk 4194304,0 > $O/ber_bin_$rep.json 2> $O/ber_bin_$rep.err || exit 1
  IBLDPC_LIB=$V/libibldpc_chloop.so timeout -k 10 400 python tools/bench_ber.py --cases c4 --batches 16 --gen-chunk 4194304,0 > $O/ber_loop_$rep.json 2> $O/ber_loop_$rep.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ber -o ber --output-format csv -- python tools/bench_ber.py --cases c4 --batches 4 > $O/bench_ber_prof.json 2> $O/bench_ber_prof.err || exit 1
