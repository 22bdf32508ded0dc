set -u
O=gpurun_out/r4f; mkdir -p $O
export TMPDIR=/tmp
(while true; do date +%T >> $O/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_float.py tests/test_gpu_ib.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed" >> $O/summary.txt; exit 1; }
echo "tests ok $(tail -1 $O/tests.log)" >> $O/summary.txt
bash tools/ab_trees.sh r4f C3 head env:IBL_FUSED_VSPLIT=0 lib:msps0 lib:st0 || exit 1
REPS=1 bash tools/ab_trees.sh r4f C1 head || exit 1
REPS=1 bash tools/ab_trees.sh r4f C2 head
