set -u
O=gpurun_out/r02p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_float.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --config C3 --no-cpu-baseline > $O/bench_C3.json 2> $O/bench_C3.err
rc=$?; echo "bench C3 rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r['kernel'], r.get('avg_launch_ms'), r['frac'])" $O/bench_C3.json 2>/dev/null)" >> $O/summary.txt
bash tools/r02o.sh
