set -u
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_float.py tests/test_gpu_encoder.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
for c in C4 C1 C2 C3 C5; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err
  rc=$?; echo "bench $c rc=$rc" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
done
