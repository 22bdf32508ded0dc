set -u
O=gpurun_out/r02f; mkdir -p $O
for c in C2 C1; do
  for pth in auto passes; do
    timeout -k 10 400 python bench.py --config $c --path $pth --no-cpu-baseline > $O/bench_${c}_$pth.json 2> $O/bench_${c}_$pth.err
    rc=$?; echo "bench $c $pth rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r['kernel'], r['avg_launch_ms'], r['frac'], r.get('lds_lookups_per_clk_per_cu'))" $O/bench_${c}_$pth.json 2>/dev/null)" >> $O/summary.txt
    [ $rc = 0 ] || exit $rc
  done
done
