#!/bin/bash
# Round-6 GPU session ah: small-batch pass chains from captured graphs: parity, lines, BER driver at B=2.
set -o pipefail
O=gpurun_out/r6ah
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_ib.py tests/test_gpu_float.py tests/test_gpu_ber_parity.py tests/test_gpu_bench_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
LINES=tools/lines_graph.txt bash tools/gpu_run.sh r6ah lines || exit 1
timeout -k 10 500 python tools/bench_ber.py --cases c4,c5 --batch 2 --batches 512 > $O/ber_b2.json 2> $O/ber_b2.err || exit 1
