#!/bin/bash
# round 6: current distilgpt2 bench + step timeline (after the hoisted-hash epilogues)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6s
mkdir -p $O
bash tools/gpu_job.sh \
  "r6s/bench:300:python -u bench.py --steps 20 --warmup 5 > $O/bench.jsonl && python -u bench.py --steps 20 --warmup 5 --epoch_lines 0 >> $O/bench.jsonl" \
  "r6s/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt"
