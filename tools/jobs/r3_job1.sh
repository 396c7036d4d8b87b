#!/bin/bash
# Round-3 first GPU pass: tests, bench (cold + warm epoch), cold-start breakdown, PMC of the step,
# P1 app [Training] epoch.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
bash tools/gpu_job.sh \
  "a_tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "a_bench:300:python bench.py" \
  "a_cold1:200:python tools/coldstart.py --steps 12" \
  "a_cold0:200:python tools/coldstart.py --steps 12 --warm_setup 0" \
  "a_p1:300:python scripts/finetune_lora_distilgpt2.py --dataset medium --logdir $O/p1_logs --out_root $O/p1_out --logging_steps 100 --step_log none && python scripts/summarize_medium_times.py $O/p1_logs" \
  "a_pmc:240:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc1 -o run -- python3 bench.py --steps 3 --warmup 1 --epoch_lines 0 && python tools/pmc_summary.py $O/pmc1 --top 30"
