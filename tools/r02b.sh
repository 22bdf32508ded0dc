set -u
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
IBL_ALLOW_SCRATCH=1 IBLDPC_LIB=$PWD/informationbottleneckdecodingldpc_amd/variants/libibldpc_spill16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ib.py -k "mixed" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/spill16.log 2>&1
rc=$?; echo "spill16 rc=$rc $(tail -1 $O/spill16.log)" >> $O/summary.txt
