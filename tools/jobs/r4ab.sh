#!/bin/bash
# round 4: LN-bwd + mask_proj one pass (one LDS exchange for both row sums) — tests, op bench, bench A/B
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4ab
mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --epoch_lines 0"
bash tools/gpu_job.sh \
  "r4ab/tests:300:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -k 'ln_bwd_mask_proj or handoff' -x -q --timeout 120 --timeout-method thread" \
  "r4ab/op:200:python tools/bench_ln_mask_proj.py --json $O/op.json" \
  "r4ab/on1:200:$B" \
  "r4ab/off1:200:MIFT_LN_MASK_PROJ=0 $B" \
  "r4ab/on2:200:$B" \
  "r4ab/off2:200:MIFT_LN_MASK_PROJ=0 $B" \
  "r4ab/on3:200:$B" \
  "r4ab/off3:200:MIFT_LN_MASK_PROJ=0 $B"
