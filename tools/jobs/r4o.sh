#!/bin/bash
# round 4: write-through in-launch LoRA wgrad slab reduction (MIFT_WGRAD_FIN=1) — tests + same-process step A/B
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4o
mkdir -p $O
bash tools/gpu_job.sh \
  "r4o/tests:300:python -u -m pytest tests/test_kernels_gpu.py -k 'wgrad or lora_proj' -x -q --timeout 120 --timeout-method thread" \
  "r4o/step_ab:600:python tools/step_ab.py 'MIFT_WGRAD_FIN=0' 'MIFT_WGRAD_FIN=1' --blocks 6 --steps 10"
