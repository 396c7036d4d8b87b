#!/bin/bash
# round 5: full GPU suite after the seq/tiled OT test fix
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r5i
bash tools/gpu_job.sh \
  "r5i/gpu_tests:1000:python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread"
