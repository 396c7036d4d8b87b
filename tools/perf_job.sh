#!/bin/bash
# GPU tests + bench + kernel-trace profile of the flagship bench (writes gpurun_out/prof_kt).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_job.sh "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "bench:300:python bench.py --steps 30 --warmup 5" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_kt -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_kt.log 2>&1
echo "prof rc=$?"
