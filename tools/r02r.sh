set -u
O=$PWD/gpurun_out/r02r; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $O/pmc1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/b1.json 2> $O/b1.err
rc=$?; echo "pmc1 rc=$rc" >> $O/summary.txt; [ $rc = 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES -d $O/pmc2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $O/b2.json 2> $O/b2.err
rc=$?; echo "pmc2 rc=$rc" >> $O/summary.txt
