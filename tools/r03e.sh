# A/B: fused IB with arithmetic task records (default) vs loaded (IBL_FUSED_UNIFORM=0) at C2/C1;
# variable-pass light row width (lw4 / lw4d2 variants) at C4. Parity tests of the fused kernel first.
set -u
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ib.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for m in 1 0; do
    IBL_FUSED_UNIFORM=$m timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline > $O/c2_u${m}_$rep.json 2> $O/c2_u${m}_$rep.err; rc=$?
    echo "C2 uniform=$m rep$rep rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline'].get('avg_launch_ms'), d['roofline']['frac'])" $O/c2_u${m}_$rep.json 2>/dev/null)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
  done
done
IBL_FUSED_UNIFORM=1 timeout -k 10 300 python bench.py --config C1 --no-cpu-baseline > $O/c1.json 2> $O/c1.err; rc=$?
echo "C1 rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'])" $O/c1.json 2>/dev/null)" >> $O/summary.txt; [ $rc = 0 ] || exit $rc

