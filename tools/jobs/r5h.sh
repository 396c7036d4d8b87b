#!/bin/bash
# round 5 checkpoint: full GPU suite, smoke, headline bench on the committed kernels
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5h
mkdir -p $O
bash tools/gpu_job.sh \
  "r5h/gpu_tests:900:python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "r5h/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r5h/bench:300:python bench.py"
