set -u
O=gpurun_out/r02q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ib.py tests/test_gpu_float.py -x -q -k "fused or random_tables or mixed or dtypes" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
for c in C2 C3 C1; do
timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
rc=$?; echo "bench $c rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r['kernel'], r.get('avg_launch_ms'), r['frac'], d['ms_per_step'])" $O/bench_$c.json 2>/dev/null)" >> $O/summary.txt
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r02q/prof_C3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C3 --no-cpu-baseline --steps 2 > /dev/null 2>&1
echo "prof rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/r02q/summary.txt
