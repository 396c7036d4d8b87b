#!/bin/bash
# round 5: GEMM raster group for the distilgpt2 block GEMMs (same-process step A/B)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5y
mkdir -p $O
bash tools/gpu_job.sh \
  "r5y/step_ab:400:python tools/step_ab.py 'MIFT_GEMM_GROUP=0' 'MIFT_GEMM_GROUP=2' 'MIFT_GEMM_GROUP=4' 'MIFT_GEMM_GROUP=8' --blocks 6 --steps 10 --json $O/step_ab_gemm_group.json"
