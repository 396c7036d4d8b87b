#!/bin/bash
# round 6: full GPU suite after the hygiene pass (removed variants), smoke, bench
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6j
mkdir -p $O
bash tools/gpu_job.sh \
  "r6j/gpu_tests:1000:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r6j/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6j/bench:300:python bench.py"
