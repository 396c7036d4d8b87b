#!/bin/bash
# round 4: whole-sequence attention forward with next-tile K-fragment prefetch (experimental build)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4j
mkdir -p $O
X="MIFT_EXT_SO=.wip/_C_exp.so"
bash tools/gpu_job.sh \
  "r4j/tests_pf:300:$X MIFT_ATTN_PF=1 python -u -m pytest tests/test_kernels_gpu.py -k 'attention or attn' -x -q --timeout 120 --timeout-method thread" \
  "r4j/a_pf0:200:$X MIFT_ATTN_PF=0 python tools/bench_attn.py" \
  "r4j/a_pf1:200:$X MIFT_ATTN_PF=1 python tools/bench_attn.py" \
  "r4j/b_pf0:200:$X MIFT_ATTN_PF=0 python tools/bench_attn.py" \
  "r4j/b_pf1:200:$X MIFT_ATTN_PF=1 python tools/bench_attn.py"
