set -u
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_float.py tests/test_gpu_ber_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
for c in C3 C5; do
timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
rc=$?; echo "bench $c rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r['kernel'], r.get('avg_ms', r.get('avg_launch_ms')), r['frac'])" $O/bench_$c.json 2>/dev/null)" >> $O/summary.txt
done
timeout -k 10 400 python bench.py --kind minsum --no-cpu-baseline --steps 3 > $O/bench_ms_dvb.json 2> $O/bench_ms_dvb.err
rc=$?; echo "bench minsum dvb rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r['kernel'], r.get('avg_ms'), r['frac'])" $O/bench_ms_dvb.json 2>/dev/null)" >> $O/summary.txt
