# Session re-entry check: full GPU tests + C4/C2 bench lines.
set -u
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_C4.json 2> $O/bench_C4.err; rc=$?; echo "C4 rc=$rc" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline > $O/bench_C2.json 2> $O/bench_C2.err; rc=$?; echo "C2 rc=$rc" >> $O/summary.txt; exit $rc
