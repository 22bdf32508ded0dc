set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r4n
(while true; do date +%T >> gpurun_out/r4n/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
CONFIGS="C4 C1 C2 C3 C5" bash tools/gpu_run.sh r4n tests smoke bench
