#!/bin/bash
# round 6: per-block phase cycles of the K = 768 distilgpt2 block GEMMs on tiles 9 / 7 / 10 / 8
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6t
mkdir -p $O
bash tools/gpu_job.sh \
  "r6t/stamps:300:python -u tools/gemm_stamps.py --shapes dgpt --tiles 9,7,10,8"
