#!/bin/bash
# round 4: tiled dK/dV occupancy A/B (MIFT_ATTN_DKDV_OCC = default / 2 / 3) at the OPT shapes
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4s
mkdir -p $O
bash tools/gpu_job.sh \
  "r4s/tests_occ2:200:MIFT_ATTN_DKDV_OCC=2 python -u -m pytest tests/test_kernels_gpu.py -k 'flash_attention_fwd_bwd or kv_len' -x -q --timeout 120 --timeout-method thread" \
  "r4s/tests_occ3:200:MIFT_ATTN_DKDV_OCC=3 python -u -m pytest tests/test_kernels_gpu.py -k 'flash_attention_fwd_bwd or kv_len' -x -q --timeout 120 --timeout-method thread" \
  "r4s/a_def:200:python tools/bench_attn.py" \
  "r4s/a_occ2:200:MIFT_ATTN_DKDV_OCC=2 python tools/bench_attn.py" \
  "r4s/a_occ3:200:MIFT_ATTN_DKDV_OCC=3 python tools/bench_attn.py" \
  "r4s/b_def:200:python tools/bench_attn.py" \
  "r4s/b_occ2:200:MIFT_ATTN_DKDV_OCC=2 python tools/bench_attn.py" \
  "r4s/b_occ3:200:MIFT_ATTN_DKDV_OCC=3 python tools/bench_attn.py"
