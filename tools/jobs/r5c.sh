#!/bin/bash
# round 5: persistent fused LM-head forward — correctness (GPU LM-head tests, bit-identity vs the one-tile
# kernel), A/B timing, and the whole step with it on / off
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5c
mkdir -p $O
bash tools/gpu_job.sh \
  "r5c/test_lm:300:python -u -m pytest tests/test_lmhead_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "r5c/bench_lm:300:python tools/bench_lm_persist.py" \
  "r5c/bench_on:200:python bench.py --steps 30 --warmup 5 --epoch_lines 0" \
  "r5c/bench_off:200:MIFT_LM_PERSIST=0 python bench.py --steps 30 --warmup 5 --epoch_lines 0" \
  "r5c/bench_on_g4:200:MIFT_GEMM_GROUP=4 python bench.py --steps 30 --warmup 5 --epoch_lines 0" \
  "r5c/bench_on2:200:python bench.py --steps 30 --warmup 5 --epoch_lines 0"
