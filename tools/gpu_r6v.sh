#!/bin/bash
# Round-6 GPU session v: fused kernels take the next phase's first ticket before the barrier: parity, A/B vs
# variant pretick0 (C3, C2, C1; two alternating repetitions), phase trace of C3 and C2.
set -o pipefail
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ib.py tests/test_gpu_float.py tests/test_gpu_bench_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for c in C3 C2 C1; do
  AB_VARIANTS="base pretick0" AB_ARGS="--config $c" bash tools/gpu_run.sh r6v_$c ab || exit 1
done
CONFIGS="C3 C2" bash tools/gpu_run.sh r6v ftrace
