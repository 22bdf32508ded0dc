# Round measurement on the GPU box: full GPU tests, bench lines of every BASELINE config (with CPU
# baselines), rocprofv3 kernel stats of each, PMC traffic of the headline. Stops at the first failure.
# usage: bash tools/measure_round.sh <tag>    (outputs under gpurun_out/<tag>/)
set -u
TAG=${1:-round}
R=$PWD
O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
step() { echo "$1 rc=$2" >> $O/summary.txt; case $2 in 0) ;; *) exit $2;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest: $(tail -1 $O/pytest.log)" >> $O/summary.txt; step pytest $rc
timeout -k 10 600 python bench.py > $O/bench_C4.json 2> $O/bench_C4.err; step bench_C4 $?
for c in C1 C2 C3 C5; do
  timeout -k 10 600 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err; step bench_$c $?
done
cd /tmp
for c in C4 C2 C3 C5; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 3 > $O/bench_prof_$c.json 2> $O/prof_$c.err
  step rocprof_$c $?
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr -d $O/pmc_$ctr -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/bench_pmc_$ctr.json 2> $O/pmc_$ctr.err
  step pmc_$ctr $?
done
echo done >> $O/summary.txt
