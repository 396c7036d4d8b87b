#!/bin/bash
# round 6: mask_positions + multi pack tests; LM dgrad rescale cost
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6i
mkdir -p $O
bash tools/gpu_job.sh \
  "r6i/tests:600:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 300 --timeout-method thread -k 'mask_positions or pack_lora_multi or opt'" \
  "r6i/lmdgrad:300:python -u tools/bench_lm_dgrad.py"
