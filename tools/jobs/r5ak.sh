#!/bin/bash
# round 5: epilogue operand prefetch on the 128-row tiles (distilgpt2 step A/B: off / aux+residual / residual only)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5ak
mkdir -p $O
bash tools/gpu_job.sh \
  "r5ak/step_ab:400:python tools/step_ab.py 'MIFT_EPI_PREFETCH=0' 'MIFT_EPI_PREFETCH=1' 'MIFT_EPI_PREFETCH=2' --blocks 6 --steps 10 --json $O/step_ab_epi_prefetch.json"
