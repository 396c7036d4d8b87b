#!/bin/bash
# round 6: full GPU suite + smoke + bench after the LM-head dgrad / lse changes
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6aa
mkdir -p $O
bash tools/gpu_job.sh \
  "r6aa/gpu_tests:1000:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r6aa/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6aa/bench:300:python bench.py > $O/bench.jsonl && python bench.py --epoch_lines 0 >> $O/bench.jsonl"
