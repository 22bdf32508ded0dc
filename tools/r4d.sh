set -u
O=gpurun_out/r4d; mkdir -p $O
export TMPDIR=/tmp
(while true; do date +%T >> $O/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_float.py tests/test_gpu_ber_parity.py tests/test_gpu_distributed.py -k "converged_codewords_h5 or world_size_invariant or rccl" -s -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/prints.log 2>&1 || exit 1
echo "prints ok" >> $O/summary.txt
bash tools/ab_trees.sh r4d C3 head lib:ieeeon || exit 1
REPS=1 bash tools/ab_trees.sh r4d C4 head env:IBL_VN_PART=heavy env:IBL_VN_PART=light
