#!/bin/bash
# GPU profiling job: kernel-trace stats + two PMC passes of the flagship bench.
# usage: bash tools/prof_job.sh [bench args...]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof
mkdir -p $O
ARGS="$@"
set -o pipefail
echo "== kernel trace"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 $ARGS > $O/kt.log 2>&1 || { echo "kt failed $?"; tail -20 $O/kt.log; exit 1; }
tail -2 $O/kt.log
echo "== pmc1"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $O/pmc1 -o run -- python3 $R/bench.py --steps 3 --warmup 1 $ARGS > $O/pmc1.log 2>&1 || { echo "pmc1 failed $?"; tail -20 $O/pmc1.log; exit 1; }
echo "== pmc2"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 $ARGS > $O/pmc2.log 2>&1 || { echo "pmc2 failed $?"; tail -20 $O/pmc2.log; exit 1; }
find $O -name "*.csv" | head -20
