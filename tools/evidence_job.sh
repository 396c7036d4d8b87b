#!/bin/bash
# BASELINE-metric evidence on one MI355X: wall-clock/epoch of the P1 app on
# medium-shaped synthetic data, the reference lab workloads with published numbers (tiny-BERT DDP
# train, greedy-generation probe), and the OPT-2.7B / OPT-6.7B single-GPU LoRA steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/evidence
mkdir -p $O
bash tools/gpu_job.sh \
  "p1_medium:300:python scripts/finetune_lora_distilgpt2.py --dataset medium --logdir $O/p1_logs --out_root $O/p1_out --logging_steps 100 --step_log none && python scripts/summarize_medium_times.py $O/p1_logs" \
  "tiny_bert:300:python labs/tiny/train_tiny.py --subset 2000 --epochs 1 --batch 8 --out $O/tiny_out --no_tb" \
  "gen_probe:200:python scripts/gen_probe.py --repeat 3" \
  "opt27b:400:python bench.py --model facebook/opt-2.7b --micro_batch 48 --steps 3 --warmup 1" \
  "opt67b:500:python bench.py --model facebook/opt-6.7b --micro_batch 24 --steps 3 --warmup 1"
