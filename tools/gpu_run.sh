#!/bin/bash
# GPU-box session: tests, bench, rocprofv3 kernel trace. Stops at the first crash-like exit.
# usage: bash tools/gpu_run.sh <tag> [tests|bench|prof|pmc ...]
set -u
TAG=${1:-run}; shift
STEPS=${@:-tests bench prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
crash() { case $1 in 124|134|137|139) echo "crash-like exit $1 in $2, stopping" | tee -a $O/summary.txt; exit $1;; esac; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -m pytest $R/tests -m gpu -q --timeout 400 -p no:cacheprovider > $O/pytest.log 2>&1
      rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; crash $rc pytest;;
    ibtests)
      timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_ib.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_ib.log 2>&1
      rc=$?; echo "pytest ib rc=$rc $(tail -1 $O/pytest_ib.log)" >> $O/summary.txt; crash $rc pytest_ib; [ $rc = 0 ] || exit $rc;;
    enctests)
      timeout -k 10 600 python -m pytest $R/tests/test_gpu_encoder.py -m gpu -x -q --timeout 300 -p no:cacheprovider > $O/pytest_enc.log 2>&1
      rc=$?; echo "pytest enc rc=$rc $(tail -1 $O/pytest_enc.log)" >> $O/summary.txt; crash $rc pytest_enc; [ $rc = 0 ] || exit $rc;;
    smoke)
      timeout -k 10 300 python -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc" >> $O/summary.txt; crash $rc smoke;;
    bench)
      timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
      rc=$?; echo "bench rc=$rc" >> $O/summary.txt; crash $rc bench;;
    ab)
      # A/B the kernel variants built by tools/variants.py (AB_VARIANTS="w1 w2 ...")
      for v in ${AB_VARIANTS:-w1 w2}; do
        IBLDPC_LIB=$R/informationbottleneckdecodingldpc_amd/variants/libibldpc_$v.so timeout -k 10 300 python $R/bench.py --no-cpu-baseline ${AB_ARGS:-} > $O/ab_$v.json 2> $O/ab_$v.err
        rc=$?; echo "ab $v rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['avg_ms'], d['decoded_bit_errors'])" $O/ab_$v.json 2>/dev/null)" >> $O/summary.txt; crash $rc ab_$v
      done;;
    bsweep)
      for b in 4096 16384 32768; do
        timeout -k 10 400 python $R/bench.py --batch-per-gpu $b --steps 3 --no-cpu-baseline > $O/bench_b$b.json 2> $O/bench_b$b.err
        rc=$?; echo "bench B=$b rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['avg_ms'])" $O/bench_b$b.json 2>/dev/null)" >> $O/summary.txt; crash $rc bsweep
      done;;
    trace)
      IBL_TRACE_WAVES=$O/trace timeout -k 10 300 python $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err
      rc=$?; echo "trace rc=$rc" >> $O/summary.txt; crash $rc trace;;
    configs)
      for c in C2 C3 C5; do
        timeout -k 10 600 python $R/bench.py --config $c --steps 3 > $O/bench_$c.json 2> $O/bench_$c.err
        rc=$?; echo "bench $c rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['avg_ms'], d['roofline']['frac'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)" $O/bench_$c.json 2>/dev/null)" >> $O/summary.txt; crash $rc bench_$c
      done;;
    mrank)
      # N>1 bench path rehearsal on one GPU: 2 ranks sharing cuda:0 over gloo
      IBL_SHARE_DEVICE=1 IBL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_2rank.json 2> $O/bench_2rank.err
      rc=$?; echo "mrank rc=$rc" >> $O/summary.txt; crash $rc mrank;;
    benchfloat)
      for k in minsum bp; do
        timeout -k 10 400 python $R/bench.py --kind $k --no-cpu-baseline --steps 3 > $O/bench_$k.json 2> $O/bench_$k.err
        rc=$?; echo "bench $k rc=$rc" >> $O/summary.txt; crash $rc bench_$k
      done;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 > $O/bench_prof.json 2> $O/prof.err)
      rc=$?; echo "rocprof rc=$rc" >> $O/summary.txt; crash $rc rocprof;;
    profc3)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 $R/bench.py --config C3 --no-cpu-baseline --steps 2 > $O/bench_prof_c3.json 2> $O/prof_c3.err)
      rc=$?; echo "rocprof C3 rc=$rc" >> $O/summary.txt; crash $rc rocprof_c3;;
    proffloat)
      for k in minsum bp; do
        (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$k -o run --output-format csv -- python3 $R/bench.py --kind $k --no-cpu-baseline --steps 2 > $O/bench_prof_$k.json 2> $O/prof_$k.err)
        rc=$?; echo "rocprof $k rc=$rc" >> $O/summary.txt; crash $rc rocprof_$k
      done;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && timeout -k 10 600 rocprofv3 --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/bench_pmc_$c.json 2> $O/pmc_$c.err)
        rc=$?; echo "pmc $c rc=$rc" >> $O/summary.txt; crash $rc pmc_$c
      done;;
    sq)
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/pmc_SQ -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/bench_pmc_sq.json 2> $O/pmc_sq.err)
      rc=$?; echo "pmc SQ rc=$rc" >> $O/summary.txt; crash $rc pmc_sq;;
    sq2)
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $O/pmc_SQ2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/bench_pmc_sq2.json 2> $O/pmc_sq2.err)
      rc=$?; echo "pmc SQ2 rc=$rc" >> $O/summary.txt; crash $rc pmc_sq2;;
  esac
done
echo done >> $O/summary.txt
