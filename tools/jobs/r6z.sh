#!/bin/bash
# round 6: LM-head lse kernel with one stats round trip per row; step timeline
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6z
mkdir -p $O
bash tools/gpu_job.sh \
  "r6z/tests:300:python -u -m pytest tests/test_lmhead_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "r6z/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt"
