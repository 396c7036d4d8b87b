#!/bin/bash
# round 5: graphed generate() host path (no eager-only uploads, remembered arena holder, eval() only when training)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5ab
mkdir -p $O
bash tools/gpu_job.sh \
  "r5ab/tests:300:python -u -m pytest tests/test_infer_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "r5ab/probe:200:python -m mift.apps.gen_probe --repeat 10 && python -m mift.apps.gen_probe --repeat 10 --prompts distinct" \
  "r5ab/kt:300:rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -m mift.apps.gen_probe --repeat 2 && python tools/gen_timeline.py $O/kt/run_kernel_trace.csv > $O/gen_timeline.txt"
