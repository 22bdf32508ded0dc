set -u
O=gpurun_out/r4c; mkdir -p $O
export TMPDIR=/tmp
# heartbeat: long pytest collections (first torch import on a fresh box) print nothing for minutes
(while true; do date +%T >> $O/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 420 python -u -m pytest tests/test_gpu_float.py -k "dataflow or fused" -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/flowtests.log 2>&1 || { echo "flowtests failed rc=$?" >> $O/summary.txt; exit 1; }
echo "flowtests ok $(tail -1 $O/flowtests.log)" >> $O/summary.txt
bash tools/ab_trees.sh r4c C3 head env:IBL_FUSED_FLOW=0 lib:noieee || exit 1
bash tools/ab_trees.sh r4c C5 tree:abtrees/r02 head lib:noieee || exit 1
bash tools/gpu_run.sh r4c tests
