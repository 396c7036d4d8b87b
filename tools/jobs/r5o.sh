#!/bin/bash
# round 5: decode attention with the first 256 keys' K/V requested up front
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5o
mkdir -p $O
bash tools/gpu_job.sh \
  "r5o/tests:300:python -u -m pytest tests/test_infer_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "r5o/probe:200:python -m mift.apps.gen_probe --repeat 5 && python -m mift.apps.gen_probe --repeat 5 --prompts distinct" \
  "r5o/kt:300:rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -m mift.apps.gen_probe --repeat 2 && python tools/gen_timeline.py $O/kt/run_kernel_trace.csv > $O/gen_timeline.txt"
