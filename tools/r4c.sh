set -u
O=gpurun_out/r4c3; mkdir -p $O
export TMPDIR=/tmp
(while true; do date +%T >> $O/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
bash tools/ab_trees.sh r4c3 C3 head lib:noieee || exit 1
REPS=1 bash tools/ab_trees.sh r4c3 C5 head || exit 1
bash tools/gpu_run.sh r4c3 tests
