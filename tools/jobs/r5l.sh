#!/bin/bash
# round 5: whole-call generate graph (prefill + all decode steps in one replay)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5l
mkdir -p $O
bash tools/gpu_job.sh \
  "r5l/tests:300:python -u -m pytest tests/test_infer_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "r5l/probe:200:python -m mift.apps.gen_probe --repeat 5 && python -m mift.apps.gen_probe --repeat 5 --prompts distinct" \
  "r5l/kt:300:rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -m mift.apps.gen_probe --repeat 2 && python tools/gen_timeline.py $O/kt/run_kernel_trace.csv > $O/gen_timeline.txt"
