set -u
for c in C2 C3 C1; do
  timeout -k 10 700 bash tools/ab_env.sh s4ab_$c "- IBLDPC_LIB=informationbottleneckdecodingldpc_amd/variants/libibldpc_tka.so IBLDPC_LIB=informationbottleneckdecodingldpc_amd/variants/libibldpc_fvd3.so IBLDPC_LIB=informationbottleneckdecodingldpc_amd/variants/libibldpc_tka3.so" --config $c || exit $?
done
