set -u
O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ib.py -x -q -k "fused or random_tables or mixed" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_ib.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest_ib.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --config C2 --no-cpu-baseline > $O/bench_C2.json 2> $O/bench_C2.err
rc=$?; echo "bench C2 rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r['kernel'], r['avg_launch_ms'], r['frac'], r.get('lds_lookups_per_clk_per_cu'))" $O/bench_C2.json 2>/dev/null)" >> $O/summary.txt
IBL_TRACE_FUSED=$O/ftrace.bin IBLDPC_LIB=$PWD/informationbottleneckdecodingldpc_amd/variants/libibldpc_ftrace.so timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline --steps 1 --warmup 0 > $O/b.json 2> $O/b.err
echo "trace rc=$?" >> $O/summary.txt
