set -u
O=gpurun_out/r4l; mkdir -p $O
export TMPDIR=/tmp
(while true; do date +%T >> $O/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
CONFIGS="C1 C2" bash tools/gpu_run.sh r4l ftrace
