#!/bin/bash
# Round-6 GPU session ab: light-first share of the C4 variable pass (IBL_MIX16 of 16 waves), 3 alternating reps.
set -o pipefail
O=gpurun_out/${TAG:-r6ab}
mkdir -p $O
V=informationbottleneckdecodingldpc_amd/variants
run() {
  local n=$1 lib=$2; shift 2
  IBLDPC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || exit 1
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], (j['roofline'] or {}).get('avg_ms'))" $O/$n.json $n >> $O/summary.txt
}
for rep in 1 2 3; do
  run base4_$rep "" --config C4
  for m in ${MIXES:-mixw3 mixw5 mixw6}; do
    run ${m}_$rep $V/libibldpc_$m.so --config C4
  done
done
