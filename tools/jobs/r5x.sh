#!/bin/bash
# round 5: v2 attention forward (32x32x16) with the XCD-aware tile mapping vs v1, OPT shapes
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5x
mkdir -p $O
bash tools/gpu_job.sh \
  "r5x/tests:300:python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k 'attention or attn or flash'" \
  "r5x/attn_ab:300:python tools/bench_attn.py --ab MIFT_ATTN_FWD=1,2 --json $O/bench_attn_fwd_v1_v2_xcd.json"
