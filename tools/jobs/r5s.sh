#!/bin/bash
# round 5: rowproj waves per block 8 vs 12 (distilgpt2 widths)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5s
mkdir -p $O
bash tools/gpu_job.sh \
  "r5s/tests12:300:MIFT_ROWPROJ_NW=12 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -v --timeout 120 --timeout-method thread -k 'rowproj or ln_bwd_mask or lora_proj_and or handoff'" \
  "r5s/step_ab:400:python tools/step_ab.py 'MIFT_ROWPROJ_NW=8' 'MIFT_ROWPROJ_NW=12' 'MIFT_ROWPROJ_NW=4' --blocks 8 --steps 10 --json $O/step_ab_rowproj_nw.json"
