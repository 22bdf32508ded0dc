# Final check of the round's tree: GPU suite, smoke(), headline bench (with CPU baseline), rocprof kernel
# stats and PMC traffic of C4, rocprof of C2, the N>1 bench path rehearsed with 2 ranks on one GPU (gloo).
set -u
R=$PWD
O=$R/gpurun_out/r03j; mkdir -p $O
export TMPDIR=/tmp
step() { echo "$1 rc=$2" >> $O/summary.txt; case $2 in 0) ;; *) exit $2;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest: $(tail -1 $O/pytest.log)" >> $O/summary.txt; step pytest $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; step smoke $?
timeout -k 10 600 python bench.py > $O/bench_C4.json 2> $O/bench_C4.err; step bench_C4 $?
timeout -k 10 600 python bench.py --config C2 > $O/bench_C2.json 2> $O/bench_C2.err; step bench_C2 $?
timeout -k 10 600 python bench.py --config C1 > $O/bench_C1.json 2> $O/bench_C1.err; step bench_C1 $?
cd /tmp
for c in C4 C2; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 3 > $O/bench_prof_$c.json 2> $O/prof_$c.err
  step rocprof_$c $?
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr -d $O/pmc_$ctr -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/bench_pmc_$ctr.json 2> $O/pmc_$ctr.err
  step pmc_$ctr $?
done
cd $R
IBL_SHARE_DEVICE=1 IBL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_2rank.json 2> $O/bench_2rank.err
step mrank $?
echo done >> $O/summary.txt
