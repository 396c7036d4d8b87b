#!/bin/bash
# round 6: in-step sweep of the grouped LoRA weight-gradient launch size (target blocks, default 2048)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ao
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ao/ab:600:python -u tools/step_ab.py 'MIFT_WGRAD_BLOCKS=2048' 'MIFT_WGRAD_BLOCKS=1024' 'MIFT_WGRAD_BLOCKS=3072' 'MIFT_WGRAD_BLOCKS=4096' --blocks 8 --steps 20 --json $O/step_ab_dgpt_wgrad_blocks.json"
