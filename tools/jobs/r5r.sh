#!/bin/bash
# round 5: 8-wave rowproj blocks at the distilgpt2 widths (A/B), tests under both forms
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5r
mkdir -p $O
bash tools/gpu_job.sh \
  "r5r/tests8:300:MIFT_ROWPROJ_NW=8 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -v --timeout 120 --timeout-method thread -k 'rowproj or ln_bwd_mask or lora_proj_and or handoff'" \
  "r5r/step_ab:400:python tools/step_ab.py 'MIFT_ROWPROJ_NW=4' 'MIFT_ROWPROJ_NW=8' --blocks 8 --steps 10 --json $O/step_ab_rowproj_nw.json" \
  "r5r/kt8:300:MIFT_ROWPROJ_NW=8 rocprofv3 --kernel-trace --output-format csv -d $O/kt8 -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt8/run_kernel_trace.csv > $O/step_timeline_nw8.txt"
