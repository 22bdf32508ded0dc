set -u
O=gpurun_out/r4e; mkdir -p $O
export TMPDIR=/tmp
(while true; do date +%T >> $O/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
IBL_VN_PART=heavy CONFIGS=C4 bash tools/gpu_run.sh r4e_heavy sq || exit 1
IBL_VN_PART=light CONFIGS=C4 bash tools/gpu_run.sh r4e_light sq || exit 1
CONFIGS=C4 bash tools/gpu_run.sh r4e_all sq || exit 1
CONFIGS="C3 C2" bash tools/gpu_run.sh r4e ftrace
