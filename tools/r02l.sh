set -u
O=gpurun_out/r02l; mkdir -p $O
IBL_TRACE_FUSED=$O/fltrace.bin IBLDPC_LIB=$PWD/informationbottleneckdecodingldpc_amd/variants/libibldpc_ftrace.so timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline --steps 1 --warmup 0 > $O/b.json 2> $O/b.err
echo "rc=$?" >> $O/summary.txt
