#!/bin/bash
# round 4: hd-80 attention staging-write order (tile_chunk), two-launch optimizer, LM-head folds
# (loss total in the lse launch, in-kernel ignore id, 1/tokens multiplier in the dgrad reduction):
# full GPU suite, bench, attention timings + LDS-conflict PMC, step timeline, eager decode trace
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4e
mkdir -p $O
bash tools/gpu_job.sh \
  "r4e/new_tests:300:python -u -m pytest tests/test_optimizer_fold_gpu.py tests/test_lmhead_gpu.py tests/test_kernels_gpu.py -k 'fold or lmhead or attention or attn or adamw or grad_stats' -x -q --timeout 120 --timeout-method thread" \
  "r4e/bench:300:python bench.py --steps 20 --warmup 5" \
  "r4e/pytest:900:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r4e/bench_attn:200:python tools/bench_attn.py --json $O/bench_attn.json" \
  "r4e/pmc_attn:120:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmcattn -o run -- python3 tools/bench_attn.py && python tools/pmc_summary.py $O/pmcattn --top 16" \
  "r4e/kt_step:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py \$(find $O/kt -name '*kernel_trace.csv' | head -1)" \
  "r4e/kt_decode:200:MIFT_GEN_GRAPH=0 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktdec -o run -- python3 scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 3"
