set -u
O=gpurun_out/r02h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ib.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_ib.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest_ib.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
for c in C2 C1; do
  for pth in auto passes; do
    timeout -k 10 400 python bench.py --config $c --path $pth --no-cpu-baseline > $O/bench_${c}_$pth.json 2> $O/bench_${c}_$pth.err
    rc=$?; echo "bench $c $pth rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r['kernel'], r['avg_launch_ms'], r['frac'], r.get('lds_lookups_per_clk_per_cu'))" $O/bench_${c}_$pth.json 2>/dev/null)" >> $O/summary.txt
    [ $rc = 0 ] || exit $rc
  done
done
