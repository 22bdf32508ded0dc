#!/bin/bash
# Round-6 GPU session aa: round 5's <= 1 % adoptions re-checked on three alternating same-box repetitions
# (VERDICT r05 #5): nontemporal check-pass rows (ntcn0), 4/16 light-first variable waves (mix0) at C4; contiguous
# small-batch task records (contig0) at B = 2 / 32 (events off).
set -o pipefail
O=gpurun_out/r6aa
mkdir -p $O
V=informationbottleneckdecodingldpc_amd/variants
run() {  # run <name> <lib or ''> <args...>
  local n=$1 lib=$2; shift 2
  IBLDPC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || exit 1
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], (j['roofline'] or {}).get('avg_ms'))" $O/$n.json $n >> $O/summary.txt
}
for rep in 1 2 3; do
  run c4_base_$rep "" --config C4
  run c4_ntcn0_$rep $V/libibldpc_ntcn0.so --config C4
  run c4_mix0_$rep $V/libibldpc_mix0.so --config C4
done
for rep in 1 2 3; do
  run b2_base_$rep "" --config C4 --batch-per-gpu 2 --steps 200 --warmup 20 --no-kernel-events
  run b2_contig0_$rep $V/libibldpc_contig0.so --config C4 --batch-per-gpu 2 --steps 200 --warmup 20 --no-kernel-events
  run b32_base_$rep "" --config C4 --batch-per-gpu 32 --steps 100 --warmup 10 --no-kernel-events
  run b32_contig0_$rep $V/libibldpc_contig0.so --config C4 --batch-per-gpu 32 --steps 100 --warmup 10 --no-kernel-events
done
