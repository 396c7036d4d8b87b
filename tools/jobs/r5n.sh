#!/bin/bash
# round 5: chunked LM head (K7) A/B + decode with pinned prologue
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5n
mkdir -p $O
bash tools/gpu_job.sh \
  "r5n/tests:300:python -u -m pytest tests/test_lmhead_gpu.py tests/test_infer_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "r5n/probe:200:python -m mift.apps.gen_probe --repeat 5 && python -m mift.apps.gen_probe --repeat 5 --prompts distinct" \
  "r5n/step_ab:500:python tools/step_ab.py 'MIFT_LM_CHUNK=0' 'MIFT_LM_CHUNK=1024' 'MIFT_LM_CHUNK=2048' 'MIFT_LM_CHUNK=4096' 'MIFT_LM_CHUNK=2048 MIFT_LM_SPLIT=8' --blocks 6 --steps 10 --json $O/step_ab_lm_chunk.json"
