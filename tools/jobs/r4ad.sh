#!/bin/bash
# round 4: LoRA weight-gradient grid size (MIFT_WGRAD_BLOCKS) on the replayed distilgpt2 step
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4ad
mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --epoch_lines 0"
bash tools/gpu_job.sh \
  "r4ad/b2048a:200:$B" \
  "r4ad/b1024a:200:MIFT_WGRAD_BLOCKS=1024 $B" \
  "r4ad/b4096a:200:MIFT_WGRAD_BLOCKS=4096 $B" \
  "r4ad/b3072a:200:MIFT_WGRAD_BLOCKS=3072 $B" \
  "r4ad/b2048b:200:$B" \
  "r4ad/b1024b:200:MIFT_WGRAD_BLOCKS=1024 $B" \
  "r4ad/b4096b:200:MIFT_WGRAD_BLOCKS=4096 $B" \
  "r4ad/b3072b:200:MIFT_WGRAD_BLOCKS=3072 $B"
