set -u
O=gpurun_out/r4c2; mkdir -p $O
export TMPDIR=/tmp
(while true; do date +%T >> $O/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
bash tools/ab_trees.sh r4c2 C5 tree:abtrees/r02 head lib:noieee || exit 1
bash tools/ab_trees.sh r4c2 C3 head lib:noieee || exit 1
bash tools/gpu_run.sh r4c2 tests
