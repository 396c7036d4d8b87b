#!/bin/bash
# round 5: OPT-2.7B dp1 mb48 (bench + epoch) and its kernel-time composition (graph replay, kernel trace only)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5v
mkdir -p $O
bash tools/gpu_job.sh \
  "r5v/opt_dp1_mb48:900:python bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 5 --warmup 2" \
  "r5v/kt_opt:400:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 3 --warmup 2 --epoch_lines 0"
