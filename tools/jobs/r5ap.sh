#!/bin/bash
# round 5 final .so: full GPU suite, smoke, bench x2, OPT-2.7B dp1 mb48 (bench + epoch)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5ap
mkdir -p $O
bash tools/gpu_job.sh \
  "r5ap/gpu_tests:1000:python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread" \
  "r5ap/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r5ap/bench1:300:python bench.py" \
  "r5ap/bench2:300:python bench.py" \
  "r5ap/opt_mb48:900:python bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 5 --warmup 2"
