# fused IB decoder with two table sets: parity tests, then C2/C1 A/B (dbuf on / off) and the fused phase trace
set -u
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ib.py -q -k "fused" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for m in 1 0; do
    IBL_FUSED_DBUF=$m timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline > $O/c2_d${m}_$rep.json 2> $O/c2_d${m}_$rep.err; rc=$?
    echo "C2 dbuf=$m rep$rep rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline'].get('avg_launch_ms'), d['roofline']['frac'])" $O/c2_d${m}_$rep.json 2>/dev/null)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
  done
done
for m in 1 0; do
  IBL_FUSED_DBUF=$m timeout -k 10 300 python bench.py --config C1 --no-cpu-baseline > $O/c1_d${m}.json 2> $O/c1_d${m}.err; rc=$?
  echo "C1 dbuf=$m rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'])" $O/c1_d${m}.json 2>/dev/null)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
done
