#!/bin/bash
# Round-3 twelfth GPU pass: attention head split (bit-identity tests, sweep, step A/B).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "m_tests:300:python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k 'attention or flash'" \
  "m_sweep:200:python tools/bench_attn.py --sweep" \
  "m_ab:400:python tools/step_ab.py 'MIFT_ATTN_SPLIT=1' 'MIFT_ATTN_SPLIT=0'"
