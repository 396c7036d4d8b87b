#!/bin/bash
# round 6: LoRA wgrad ordered reduce with all column groups' slab loads in flight; step A/B vs previous build is
# not possible in one process, so: the wgrad tests + a step timeline
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ae
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ae/tests:600:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread -k 'wgrad or lora'" \
  "r6ae/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt"
