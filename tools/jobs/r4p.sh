#!/bin/bash
# round 4: OPT-2.7B dp1 at the planner's PP micro-batch (12): kernel trace of graph-replayed steps
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4p
mkdir -p $O
bash tools/gpu_job.sh \
  "r4p/kt_opt_mb12:400:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 2 --warmup 1 --out $O/mb12.jsonl && python tools/prof_summary.py $O/kt --top 40 > $O/kt_summary.txt"
