set -u
O=gpurun_out/r4r; mkdir -p $O
export TMPDIR=/tmp
(while true; do date +%T >> $O/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_float.py tests/test_gpu_ber_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed" >> $O/summary.txt; exit 1; }
echo "tests ok $(tail -1 $O/tests.log)" >> $O/summary.txt
REPS=3 bash tools/ab_trees.sh r4r C3 head lib:old || exit 1
