#!/bin/bash
# round 6: per-block phase cycles of the distilgpt2 block GEMMs with / without the LoRA K-extension
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6at
mkdir -p $O
bash tools/gpu_job.sh \
  "r6at/stamps:300:python -u tools/gemm_stamps.py --shapes dgpt --tiles 9,7 --ext" \
  "r6at/stamps_bias:300:python -u tools/gemm_stamps.py --shapes dgpt --tiles 9,7 --ext --bias > gpurun_out/r6at/stamps_bias.txt"
