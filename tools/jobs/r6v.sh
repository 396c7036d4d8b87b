#!/bin/bash
# round 6: LM-head shapes on tile 8 / tile 10 / hipBLASLt incl. the split-K proxy of the dgrad
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6v
mkdir -p $O
bash tools/gpu_job.sh \
  "r6v/lm:300:python -u tools/bench_gemm4.py --only lm_head --json $O/bench_lm_shapes.json"
