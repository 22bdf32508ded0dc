set -u
O=gpurun_out/r4s; mkdir -p $O
export TMPDIR=/tmp
(while true; do date +%T >> $O/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
bash tools/gpu_run.sh r4s mrank || exit 1
for c in C3 C5; do
  IBL_SHARE_DEVICE=1 IBL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --config $c --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_2rank_$c.json 2> $O/bench_2rank_$c.err
  rc=$?; echo "mrank $c rc=$rc" >> $O/summary.txt; [ $rc -eq 0 ] || exit $rc
done
