#!/bin/bash
# round 6: OPT-2.7B mb12 in-step knob sweep (epilogue operand groups, raster group, NT stores)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6as
mkdir -p $O
bash tools/gpu_job.sh \
  "r6as/ab:800:python -u tools/step_ab.py 'X=0' 'MIFT_EPI_PFG=0' 'MIFT_GEMM_GROUP=4' 'MIFT_GEMM_GROUP=8' 'MIFT_EPI_NT=1' --model opt-2.7b --blocks 4 --steps 3 --json $O/step_ab_opt_knobs.json"
