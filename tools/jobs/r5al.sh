#!/bin/bash
# round 5: the eight OPT-2.7B layer GEMMs at M = 6144 / 24576 against hipBLASLt (torch.matmul), auto tile
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5al
mkdir -p $O
bash tools/gpu_job.sh \
  "r5al/opt_blas:400:TILES=0 python -u tools/bench_kernels.py --only opt_blas --json $O/bench_opt_vs_hipblaslt.json"
