#!/bin/bash
# round 6: in-step sweep of the block-GEMM tile raster group (default: row panels, g = 0, below N = 8192)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6an
mkdir -p $O
bash tools/gpu_job.sh \
  "r6an/ab:600:python -u tools/step_ab.py 'MIFT_GEMM_GROUP=0' 'MIFT_GEMM_GROUP=2' 'MIFT_GEMM_GROUP=4' 'MIFT_GEMM_GROUP=8' --blocks 8 --steps 20 --json $O/step_ab_dgpt_gemm_group.json"
