# C3 on the standard 802.11n Z=81 code: the tests that use it + the C3 bench line (with CPU baseline).
set -u
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_float.py tests/test_gpu_ber_parity.py tests/test_gpu_encoder.py tests/test_gpu_ib.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C3 > $O/bench_C3.json 2> $O/bench_C3.err; rc=$?; echo "C3 rc=$rc" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
IBL_TRACE_WAVES=$O/trace timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err; rc=$?; echo "trace rc=$rc" >> $O/summary.txt; exit $rc
