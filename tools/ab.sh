# A/B of kernel variants on one box: bash tools/ab.sh <tag> "<variant ...>" [bench args]
# "base" = the default in-tree build; others = informationbottleneckdecodingldpc_amd/variants/libibldpc_<v>.so
set -u
TAG=$1; VARS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for v in $VARS; do
    if [ $v = base ]; then LIBV=""; else LIBV=$PWD/informationbottleneckdecodingldpc_amd/variants/libibldpc_$v.so; fi
    IBLDPC_LIB=$LIBV timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err
    rc=$?
    echo "$v rep$rep rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r.get('avg_ms'), d['decoded_bit_errors'])" $O/ab_${v}_$rep.json 2>/dev/null)" >> $O/summary.txt
    [ $rc = 0 ] || exit $rc
  done
done
