# PMC passes over tools/diag_lmhead.py (fused LM-head forward vs plain GEMM), one rocprofv3 run per pass
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmclm
mkdir -p $O
export DIAG_QUICK=1 MIFT_LM_DBG=0
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $O/p1 -o run -- python3 $R/tools/diag_lmhead.py > $O/p1.log 2>&1 || { echo "p1 failed $?"; tail -5 $O/p1.log; exit 1; }
echo p1 ok
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2 -o run -- python3 $R/tools/diag_lmhead.py > $O/p2.log 2>&1 || { echo "p2 failed $?"; tail -5 $O/p2.log; exit 1; }
echo p2 ok
