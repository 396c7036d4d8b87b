#!/bin/bash
# round 6: K sweep (per-tile overhead vs per-k-tile loop time) + PMC of tile 10 vs tile 8 on one shape
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 400 python -u tools/bench_gemm4.py --sweep --json $O/sweep.json > $O/sweep.log 2>&1 && \
cd /tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $GRAFT_REPO_ROOT/$O/p1 -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_gemm4.py > $GRAFT_REPO_ROOT/$O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_MFMA --output-format csv -d $GRAFT_REPO_ROOT/$O/p2 -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_gemm4.py > $GRAFT_REPO_ROOT/$O/p2.log 2>&1
