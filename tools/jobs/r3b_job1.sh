#!/bin/bash
# Round-3 (session 2) validation of the restored tree: GPU tests, smoke, driver-style bench, kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
bash tools/gpu_job.sh \
  "b_tests:500:python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread" \
  "b_smoke:150:python __graft_entry__.py smoke" \
  "b_bench:200:python bench.py" \
  "b_kt:240:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0"
