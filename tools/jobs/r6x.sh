#!/bin/bash
# round 6: row-stride effect on the LM-head dgrad proxy
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6x
mkdir -p $O
bash tools/gpu_job.sh \
  "r6x/stride:300:python -u tools/bench_lm_stride.py"
