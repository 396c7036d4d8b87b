#!/bin/bash
# round 6: LM-head dgrad over the split-K count (window tails), before the window-size change
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6w
mkdir -p $O
bash tools/gpu_job.sh \
  "r6w/lmd:300:python -u tools/bench_lm_dgrad.py"
