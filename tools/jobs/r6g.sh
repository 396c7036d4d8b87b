#!/bin/bash
# round 6: kernel traces of the distilgpt2 step and the OPT mb48 step (graph replay)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6g
mkdir -p $O
bash tools/gpu_job.sh \
  "r6g/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt" \
  "r6g/kt_opt:600:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kto -o run -- python3 bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 3 --warmup 2 --epoch_lines 0 && python tools/prof_summary.py $O/kto/run_kernel_stats.csv > $O/kernel_stats_opt.txt"
