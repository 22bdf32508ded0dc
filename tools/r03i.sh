# fused float phase trace at C3 (per-wave done clocks and task counts) and fused IB trace at C2
set -u
O=gpurun_out/r03i; mkdir -p $O
L=$PWD/informationbottleneckdecodingldpc_amd/variants/libibldpc_ftrace.so
IBL_TRACE_FUSED=$O/fltrace_c3.bin IBLDPC_LIB=$L timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline --steps 1 --warmup 0 > $O/b3.json 2> $O/b3.err; rc=$?
echo "trace C3 rc=$rc" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
IBL_TRACE_FUSED=$O/ftrace_c2.bin IBLDPC_LIB=$L timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline --steps 1 --warmup 0 > $O/b2.json 2> $O/b2.err; rc=$?
echo "trace C2 rc=$rc" >> $O/summary.txt; exit $rc
