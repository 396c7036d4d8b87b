#!/bin/bash
# round 6 final tree (bias staging): decode probe, distilgpt2 step kernel trace, OPT-2.7B dp1 mb48
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ay
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ay/probe:200:python -m mift.apps.gen_probe --repeat 10 > $O/gen_probe.txt 2>&1 && python -m mift.apps.gen_probe --repeat 10 --prompts distinct >> $O/gen_probe.txt 2>&1" \
  "r6ay/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt && python tools/prof_summary.py $O/kt 13 > $O/kernel_summary.txt" \
  "r6ay/opt_mb48:900:python bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 5 --warmup 2 > $O/opt_mb48.jsonl"
