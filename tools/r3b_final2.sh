#!/bin/bash
# Round-3 (session 2) evidence, part 2: P1 app epoch, cold start, OPT-2.7B single GPU, generation probe,
# attention and LM-head micro-benchmarks.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r3bf
mkdir -p $O
bash tools/gpu_job.sh \
  "g_p1:300:python scripts/finetune_lora_distilgpt2.py --dataset medium --logdir $O/p1_logs --out_root $O/p1_out --logging_steps 100 --step_log none && python scripts/summarize_medium_times.py $O/p1_logs" \
  "g_cold:150:python tools/coldstart.py --steps 12" \
  "g_opt27b:300:python bench.py --model facebook/opt-2.7b --micro_batch 48 --steps 3 --warmup 1" \
  "g_gen:150:python scripts/gen_probe.py --prompts distinct --repeat 3" \
  "g_attn:150:python tools/bench_attn.py" \
  "g_lmhead:150:python tools/bench_lmhead.py"
