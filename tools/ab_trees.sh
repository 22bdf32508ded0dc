#!/bin/bash
# Same-box A/B of whole trees and library variants on one bench config, alternating repetitions.
# usage: bash tools/ab_trees.sh <tag> <config> <arm ...>
#   arm = "head" (this tree), "tree:<dir>" (another checkout under abtrees/, its own bench.py and .so),
#         "lib:<variant>" (this tree's bench with informationbottleneckdecodingldpc_amd/variants/libibldpc_<variant>.so)
#         or "env:<VAR>=<value>" (this tree's bench with that environment variable)
# env: REPS (default 2), AB_ARGS (extra bench args)
set -u
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for arm in "$@"; do
    name=$(echo $arm | tr ':/=' '___')
    ev=""
    case $arm in
      head)   cmd="python $R/bench.py"; lib="";;
      env:*)  cmd="python $R/bench.py"; lib=""; ev=${arm#env:};;
      tree:*) cmd="python $R/${arm#tree:}/bench.py"; lib="";;
      lib:*)  cmd="python $R/bench.py"; lib=$R/informationbottleneckdecodingldpc_amd/variants/libibldpc_${arm#lib:}.so;;
    esac
    env IBLDPC_LIB=$lib $ev timeout -k 10 300 $cmd --config $CFG --no-cpu-baseline ${AB_ARGS:-} > $O/${CFG}_${name}_$rep.json 2> $O/${CFG}_${name}_$rep.err
    rc=$?
    v=$(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r.get('avg_ms'), r.get('frac'))" $O/${CFG}_${name}_$rep.json 2>/dev/null)
    echo "$CFG $arm rep$rep rc=$rc $v" >> $O/summary.txt
    [ $rc -eq 0 ] || exit $rc
  done
done
