set -u
O=gpurun_out/r02t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ib.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
bash tools/ab.sh ab_ld "base ld2"
