# Round measurement on the GPU box: full GPU tests, smoke(), bench lines of every BASELINE config (with CPU
# baselines), rocprofv3 kernel stats of each, PMC traffic of the per-pass configs (C4, C5).
# usage: bash tools/measure_round.sh <tag>    (outputs under gpurun_out/<tag>/)
set -u
TAG=${1:-round}
CONFIGS="C4 C1 C2 C3 C5" bash tools/gpu_run.sh $TAG tests smoke bench prof || exit $?
CONFIGS="C4 C5" bash tools/gpu_run.sh $TAG pmc
