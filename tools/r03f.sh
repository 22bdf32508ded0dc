# A/B at C4: variable-pass light items with 1-KiB row segments (lw4: 3 in flight, lw4d2: 2)
set -u
O=gpurun_out/r03f; mkdir -p $O
L=$PWD/informationbottleneckdecodingldpc_amd/variants
IBLDPC_LIB=$L/libibldpc_lw4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ib.py -q -k "random_tables or mixed" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest(lw4) rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
bash tools/ab.sh r03f "base lw4 lw4d2"
