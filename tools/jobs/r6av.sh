#!/bin/bash
# round 6: bias row staged into LDS with the K-extension operands: tests, stamps, step A/B
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6av
mkdir -p $O
bash tools/gpu_job.sh \
  "r6av/tests:600:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "r6av/stamps:300:python -u tools/gemm_stamps.py --shapes dgpt --tiles 9,7 --ext --bias" \
  "r6av/ab:600:python -u tools/step_ab.py 'MIFT_EXT_LDS=0' 'MIFT_EXT_LDS=1' --blocks 8 --steps 20 --json $O/step_ab_dgpt_ext_bias_lds.json"
