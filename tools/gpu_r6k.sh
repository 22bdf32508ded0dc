#!/bin/bash
# Round-6 GPU session k: float small-batch kernels (one codeword per lane, contiguous tasks): parity, A/B lines.
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_float.py tests/test_gpu_bench_paths.py tests/test_gpu_ber_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
LINES=tools/lines_nc1.txt bash tools/gpu_run.sh r6k lines
