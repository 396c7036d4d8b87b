#!/bin/bash
# round 6: distilgpt2 step A/B: one-chip-wave N = 768 GEMMs on the 128x96 tile (default) vs the 8-wave 128x192 tile
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ah
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ah/ab:600:python -u tools/step_ab.py 'MIFT_GEMM_T96=7' 'MIFT_GEMM_T96=9' --blocks 6 --steps 20 --json $O/step_ab_dgpt_t96.json"
