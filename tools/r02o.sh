set -u
O=gpurun_out/r02o; mkdir -p $O
for b in 512 1024 2048 8192; do
  timeout -k 10 300 python bench.py --batch-per-gpu $b --no-cpu-baseline --steps 5 > $O/bench_b$b.json 2> $O/bench_b$b.err
  rc=$?; echo "B=$b rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r.get('avg_ms'), d['ms_per_step'])" $O/bench_b$b.json 2>/dev/null)" >> $O/summary.txt
  [ $rc = 0 ] || exit $rc
done
