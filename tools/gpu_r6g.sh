#!/bin/bash
# Round-6 GPU session g: the C ABI communicator test, smoke, small-batch lines (packed small-batch rows).
set -o pipefail
O=gpurun_out/r6g2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
LINES=tools/lines_small.txt bash tools/gpu_run.sh r6g2 smoke lines
