set -u
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ber_parity.py tests/test_gpu_ib.py -k "ber or full_size" -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
timeout -k 10 400 python bench.py --config C3 > $O/bench_C3.json 2> $O/bench_C3.err
rc=$?; echo "bench C3 rc=$rc" >> $O/summary.txt
