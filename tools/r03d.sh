# fused IB phase trace at C2 (two table sets) and C1
set -u
O=gpurun_out/r03d; mkdir -p $O
L=$PWD/informationbottleneckdecodingldpc_amd/variants/libibldpc_ftrace.so
IBL_TRACE_FUSED=$O/ftrace_c2.bin IBLDPC_LIB=$L timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline --steps 1 --warmup 0 > $O/b.json 2> $O/b.err; rc=$?
echo "trace rc=$rc" >> $O/summary.txt; exit $rc
