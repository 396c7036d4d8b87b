#!/bin/bash
# round 4: OPT PP micro-batch GEMM shapes (M = 2048 / 6144) over every candidate tile
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4w
mkdir -p $O
bash tools/gpu_job.sh \
  "r4w/optpp:600:TILES=0,1,3,5,6,7,8,20,21 python tools/bench_kernels.py --only optm_pp --json $O/optpp.json"
