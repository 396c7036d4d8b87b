#!/bin/bash
# round 6: LM-head dgrad window fill batched + one window per distilgpt2 chunk
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6y
mkdir -p $O
bash tools/gpu_job.sh \
  "r6y/tests:300:python -u -m pytest tests/test_lmhead_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "r6y/lmd:300:python -u tools/bench_lm_dgrad.py" \
  "r6y/bench:300:python -u bench.py --steps 20 --warmup 5 --epoch_lines 0 > $O/bench.jsonl"
