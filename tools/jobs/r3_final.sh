#!/bin/bash
# Round-3 end evidence on one MI355X: GPU tests, smoke, the driver-style bench (+ cold epoch), a kernel
# trace and a PMC pass of the flagship step, attention / LM-head / row-projection micro-benchmarks,
# OPT-2.7B single-GPU, the P1 app epoch, cold start, generation probe (padded, distinct prompts).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r3final
mkdir -p $O
bash tools/gpu_job.sh \
  "z_tests:600:python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread" \
  "z_smoke:200:python __graft_entry__.py smoke" \
  "z_bench:300:python bench.py" \
  "z_kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0" \
  "z_pmc:240:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 3 --warmup 1 --epoch_lines 0" \
  "z_attn:200:python tools/bench_attn.py" \
  "z_lmhead:200:python tools/bench_lmhead.py" \
  "z_opt27b:400:python bench.py --model facebook/opt-2.7b --micro_batch 48 --steps 3 --warmup 1" \
  "z_p1:300:python scripts/finetune_lora_distilgpt2.py --dataset medium --logdir $O/p1_logs --out_root $O/p1_out --logging_steps 100 --step_log none && python scripts/summarize_medium_times.py $O/p1_logs" \
  "z_cold:200:python tools/coldstart.py --steps 12" \
  "z_gen:200:python scripts/gen_probe.py --prompts distinct --repeat 3"
