#!/bin/bash
# GPU-box session: every measurement the rounds use, as named steps. Stops at the first failure.
# usage: bash tools/gpu_run.sh <tag> <step ...>        (outputs under gpurun_out/<tag>/)
# env:   CONFIGS="C4 C3 C2"   configs for the per-config steps (bench, prof, sq, sq2, pmc, ftrace)
#        AB_VARIANTS="base v1" variants for `ab` (tools/variants.py builds them), AB_ARGS bench args
#        BATCHES="512 4096"    batches for `bsweep`
# steps: tests ibtests floattests smoke bench prof sq sq2 pmc bsweep ab trace ftrace mrank
set -u
TAG=${1:-run}; shift
STEPS=${@:-tests bench prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
CONFIGS=${CONFIGS:-C4}
VL=$R/informationbottleneckdecodingldpc_amd/variants
# any non-zero exit ends the session (a crash-like one is labelled as such)
chk() {
  case $1 in 0) return 0;; 124|134|137|139) echo "crash-like exit $1 in $2, stopping" >> $O/summary.txt;; esac
  echo "$2 failed rc=$1" >> $O/summary.txt; exit $1
}
jf() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r.get('avg_ms'), r.get('frac'), d['decoded_bit_errors'], (d.get('cpu_baseline') or {}).get('value'))" $1 2>/dev/null; }
pmc() {  # pmc <outdir-name> <config> <counters...>: one rocprofv3 counter pass over one bench step
  local n=$1 c=$2; shift 2
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc "$@" -d $O/$n -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 1 --warmup 0 > $O/$n.json 2> $O/$n.err)
  chk $? $n; echo "$n ok" >> $O/summary.txt
}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest $R/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
      rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; chk $rc pytest;;
    ibtests|floattests)
      f=test_gpu_ib.py; [ $s = floattests ] && f="test_gpu_float.py test_gpu_ber_parity.py"
      (cd $R/tests && timeout -k 10 600 python -u -m pytest $f -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider) > $O/pytest_$s.log 2>&1
      rc=$?; echo "$s rc=$rc $(tail -1 $O/pytest_$s.log)" >> $O/summary.txt; chk $rc $s;;
    smoke)
      timeout -k 10 300 python -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc" >> $O/summary.txt; chk $rc smoke;;
    bench)
      for c in $CONFIGS; do
        timeout -k 10 600 python $R/bench.py --config $c ${BENCH_ARGS:-} > $O/bench_$c.json 2> $O/bench_$c.err
        rc=$?; echo "bench $c rc=$rc $(jf $O/bench_$c.json)" >> $O/summary.txt; chk $rc bench_$c
      done;;
    prof)
      for c in $CONFIGS; do
        (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 3 > $O/bench_prof_$c.json 2> $O/prof_$c.err)
        rc=$?; echo "rocprof $c rc=$rc" >> $O/summary.txt; chk $rc rocprof_$c
      done;;
    sq)    # LDS and issue counters (one pass: 8 SQ + 1 GRBM)
      for c in $CONFIGS; do
        pmc sq_$c $c SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
      done;;
    sq2)   # wave-state split
      for c in $CONFIGS; do
        pmc sq2_$c $c SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
      done;;
    pmc)   # HBM bytes: FETCH_SIZE and WRITE_SIZE in separate passes
      for c in $CONFIGS; do
        pmc pmc_FETCH_SIZE_$c $c FETCH_SIZE
        pmc pmc_WRITE_SIZE_$c $c WRITE_SIZE
      done;;
    bsweep)
      for b in ${BATCHES:-4096 16384}; do
        timeout -k 10 400 python $R/bench.py --batch-per-gpu $b --steps 3 --no-cpu-baseline > $O/bench_b$b.json 2> $O/bench_b$b.err
        rc=$?; echo "bench B=$b rc=$rc $(jf $O/bench_b$b.json)" >> $O/summary.txt; chk $rc bsweep
      done;;
    ab)    # A/B of kernel variants, two alternating repetitions
      for rep in 1 2; do
        for v in ${AB_VARIANTS:-base}; do
          LIBV=""; [ $v = base ] || LIBV=$VL/libibldpc_$v.so
          IBLDPC_LIB=$LIBV timeout -k 10 300 python $R/bench.py --no-cpu-baseline ${AB_ARGS:-} > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err
          rc=$?; echo "ab $v rep$rep rc=$rc $(jf $O/ab_${v}_$rep.json)" >> $O/summary.txt; chk $rc ab_$v
        done
      done;;
    trace)   # per-wave clocks of the per-pass IB kernels (tools/wave_balance.py)
      IBL_TRACE_WAVES=$O/trace IBLDPC_LIB=$VL/libibldpc_diag.so timeout -k 10 300 python $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err
      chk $? trace; echo "trace ok" >> $O/summary.txt;;
    ftrace)  # fused-kernel phase trace (variant `ftrace`; tools/fused_trace.py, tools/fused_trace_fl.py)
      for c in $CONFIGS; do
        IBL_ALLOW_SCRATCH=1 IBL_TRACE_FUSED=$O/ftrace_$c.bin IBLDPC_LIB=$VL/libibldpc_ftrace.so timeout -k 10 300 python $R/bench.py --config $c --no-cpu-baseline --steps 1 --warmup 0 > $O/ftrace_$c.json 2> $O/ftrace_$c.err
        chk $? ftrace_$c; echo "ftrace $c ok" >> $O/summary.txt
      done;;
    lines)   # one run per line of $LINES: "<name> [VAR=value ...] <command ...>" (relative paths from the repo root)
      while read -r name args; do
        [ -z "$name" ] && continue
        case $name in \#*) continue;; esac
        eval "timeout -k 10 300 env $args" > $O/line_$name.json 2> $O/line_$name.err
        rc=$?; echo "line $name rc=$rc $(jf $O/line_$name.json)" >> $O/summary.txt; chk $rc line_$name
      done < ${LINES:-tools/lines_default.txt};;
    mrank)   # N>1 bench path rehearsed on one GPU: 2 ranks sharing cuda:0 over gloo
      IBL_SHARE_DEVICE=1 IBL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline ${MRANK_ARGS:-} > $O/bench_2rank.json 2> $O/bench_2rank.err
      rc=$?; echo "mrank rc=$rc" >> $O/summary.txt; chk $rc mrank;;
    *) echo "unknown step $s" >> $O/summary.txt; exit 2;;
  esac
done
echo done >> $O/summary.txt
