#!/bin/bash
# round 4: GEMM tile experiments from the experimental build (.wip/_C_exp.so) on the distilgpt2 and OPT
# micro-batch shapes with their training epilogues
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r4c
bash tools/gpu_job.sh \
  "r4c/dgpt_tiles:400:MIFT_EXT_SO=.wip/_C_exp.so TILES=0,7,9,10,11,12 python tools/bench_kernels.py --only dgpt --json gpurun_out/r4c/dgpt_tiles.json" \
  "r4c/optm_tiles:600:MIFT_EXT_SO=.wip/_C_exp.so TILES=0,3,6,8,10,11,12 python tools/bench_kernels.py --only optm --json gpurun_out/r4c/optm_tiles.json"
