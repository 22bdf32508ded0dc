#!/bin/bash
# Round-6 GPU session o: float kernels read the grid size from the kernarg segment: parity, small-batch A/B, C3/C5.
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_float.py tests/test_gpu_bench_paths.py tests/test_gpu_ber_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
LINES=tools/lines_nc1.txt bash tools/gpu_run.sh r6o lines
