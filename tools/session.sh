#!/bin/bash
# One GPU-box session (the command a gpurun call runs): a heartbeat file so gpurun sees progress during long
# steps, then tools/gpu_run.sh with the given steps. Per-session settings go in the environment
# (CONFIGS, AB_VARIANTS, AB_ARGS, BENCH_ARGS, BATCHES — see tools/gpu_run.sh).
# usage: bash tools/session.sh <tag> <step ...>        e.g. CONFIGS="C4 C5" bash tools/session.sh r5a tests bench prof
set -u
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
(while true; do date +%T >> gpurun_out/$TAG/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
bash tools/gpu_run.sh $TAG "$@"
