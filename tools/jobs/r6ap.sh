#!/bin/bash
# round 6: where one decode step goes (kernel trace of the generation probe)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ap
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ap/kt:300:rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -m mift.apps.gen_probe --repeat 2 && python tools/decode_step_kernels.py $O/kt/run_kernel_trace.csv > $O/decode_step.txt"
