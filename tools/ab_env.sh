# A/B of environment settings on one box, two alternating repetitions:
#   bash tools/ab_env.sh <tag> "<NAME=VAL[,NAME=VAL]> ..." [bench args]     ("-" = no setting)
set -u
TAG=$1; SETS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  for s in $SETS; do
    envs=""; [ "$s" = "-" ] || envs=$(echo $s | tr ',' ' ')
    n=$(echo $s | tr -c 'A-Za-z0-9_\n' '_')
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/ab_${n}_$rep.json 2> $O/ab_${n}_$rep.err
    rc=$?
    echo "$s rep$rep rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r.get('avg_ms'), r.get('frac'), d['decoded_bit_errors'])" $O/ab_${n}_$rep.json 2>/dev/null)" >> $O/summary.txt
    [ $rc = 0 ] || exit $rc
  done
done
