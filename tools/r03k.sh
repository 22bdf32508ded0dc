# final-table slot added once per node (lane4f): IB parity tests, then A/B vs the previous build at C4 and C2
set -u
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ib.py tests/test_gpu_ber_parity.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
bash tools/ab.sh r03k "base pre" || exit $?
bash tools/ab.sh r03k_c2 "base pre" --config C2
