set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r4u
(while true; do date +%T >> gpurun_out/r4u/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
bash tools/gpu_run.sh r4u tests smoke
