#!/bin/bash
# round 6 final tree: full GPU suite, smoke, bench x2
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ax
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ax/gpu_tests:1000:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "r6ax/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6ax/bench:300:python bench.py > $O/bench.jsonl && python bench.py >> $O/bench.jsonl"
