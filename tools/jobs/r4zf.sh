#!/bin/bash
# round 4 final state check: GPU suite, smoke, bench
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4zf
mkdir -p $O
bash tools/gpu_job.sh \
  "r4zf/pytest:900:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r4zf/smoke:200:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "r4zf/bench:300:python bench.py --steps 20 --warmup 5" \
  "r4zf/bench2:300:python bench.py --steps 20 --warmup 5"
