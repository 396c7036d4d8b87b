#!/bin/bash
# round 5: greedy-decode time breakdown (prefill vs replays) for the decode target
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5j
mkdir -p $O
bash tools/gpu_job.sh \
  "r5j/probe:200:python -m mift.apps.gen_probe --repeat 5 && python -m mift.apps.gen_probe --repeat 5 --prompts distinct" \
  "r5j/kt:300:rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -m mift.apps.gen_probe --repeat 2 && python tools/gen_timeline.py $O/kt/run_kernel_trace.csv > $O/gen_timeline.txt"
