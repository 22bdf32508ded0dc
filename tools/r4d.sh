set -u
O=gpurun_out/r4d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_float.py tests/test_gpu_ber_parity.py -k "converged_codewords_h5 or world_size_invariant" -s -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/prints.log 2>&1 || exit 1
bash tools/ab_trees.sh r4d C4 head env:IBL_VN_PART=heavy env:IBL_VN_PART=light || exit 1
IBL_VN_PART=heavy CONFIGS=C4 bash tools/gpu_run.sh r4d_heavy sq || exit 1
IBL_VN_PART=light CONFIGS=C4 bash tools/gpu_run.sh r4d_light sq || exit 1
CONFIGS=C4 bash tools/gpu_run.sh r4d_all sq || exit 1
CONFIGS="C2 C1" bash tools/gpu_run.sh r4d bench || exit 1
CONFIGS="C3 C2" bash tools/gpu_run.sh r4d ftrace
