#!/bin/bash
# Round-end evidence on one MI355X: GPU tests, smoke, the driver-style bench, a kernel trace of the
# flagship step, the LM-head fused-vs-library and attention micro-benchmarks, OPT-2.7B, and the
# reference-metric apps (P1 medium epoch, tiny-BERT lab, greedy-generation probe).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
bash tools/gpu_job.sh \
  "f_tests:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "f_smoke:200:python __graft_entry__.py smoke" \
  "f_bench:240:python bench.py" \
  "f_kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0" \
  "f_lmhead:200:python tools/bench_lmhead.py" \
  "f_attn:200:python tools/bench_attn.py" \
  "f_opt27b:400:python bench.py --model facebook/opt-2.7b --micro_batch 48 --steps 3 --warmup 1" \
  "f_p1:300:python scripts/finetune_lora_distilgpt2.py --dataset medium --logdir $O/p1_logs --out_root $O/p1_out --logging_steps 100 --step_log none && python scripts/summarize_medium_times.py $O/p1_logs" \
  "f_tiny:300:python labs/tiny/train_tiny.py --subset 2000 --epochs 1 --batch 8 --out $O/tiny_out --no_tb" \
  "f_gen:200:python scripts/gen_probe.py --repeat 3"
