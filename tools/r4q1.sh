set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r4q
(while true; do date +%T >> gpurun_out/r4q/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
CONFIGS="C4 C1 C2 C3 C5" bash tools/gpu_run.sh r4q tests smoke bench || exit 1
timeout -k 10 300 python tools/bench_encoder.py > gpurun_out/r4q/encoder.json 2> gpurun_out/r4q/encoder.err && echo "encoder ok" >> gpurun_out/r4q/summary.txt
