set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r4q
(while true; do date +%T >> gpurun_out/r4q/heartbeat2; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
CONFIGS="C4 C1 C2 C3 C5" bash tools/gpu_run.sh r4q prof || exit 1
CONFIGS="C4 C5" bash tools/gpu_run.sh r4q pmc || exit 1
CONFIGS="C1 C2 C3 C4" bash tools/gpu_run.sh r4q sq || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4q/prof_enc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_encoder.py --steps 5 > $GRAFT_REPO_ROOT/gpurun_out/r4q/encoder_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r4q/encoder_prof.err) && echo "encoder prof ok" >> gpurun_out/r4q/summary.txt
