export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmcattn
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $O/p1 -o run -- python3 $R/tools/bench_attn.py > $O/p1.log 2>&1 || { echo "p1 failed $?"; tail -5 $O/p1.log; exit 1; }
echo p1 ok
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_MFMA --output-format csv -d $O/p2 -o run -- python3 $R/tools/bench_attn.py > $O/p2.log 2>&1 || { echo "p2 failed $?"; tail -5 $O/p2.log; exit 1; }
echo p2 ok
