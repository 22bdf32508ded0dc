set -u
O=gpurun_out/r4f; mkdir -p $O
export TMPDIR=/tmp
(while true; do date +%T >> $O/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_float.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/floattests.log 2>&1 || { echo "floattests failed" >> $O/summary.txt; exit 1; }
echo "floattests ok $(tail -1 $O/floattests.log)" >> $O/summary.txt
bash tools/ab_trees.sh r4f C3 head lib:msps0 lib:st0
