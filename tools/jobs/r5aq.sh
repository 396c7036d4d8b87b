#!/bin/bash
# round 5: full OPT-2.7B mb48 bench, non-temporal C stores off / default / off (same box)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5aq
mkdir -p $O
B="python bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 5 --warmup 2 --epoch_lines 0"
bash tools/gpu_job.sh "r5aq/nt0a:300:MIFT_EPI_NT=0 $B" "r5aq/ntd:300:$B" "r5aq/nt0b:300:MIFT_EPI_NT=0 $B" "r5aq/dgpt:200:python bench.py --epoch_lines 0"
