#!/bin/bash
# Round-3 tenth GPU pass: LM-head nontemporal E store / load A/B; lora_proj on the rowproj MFMA form.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "k_tests:300:python -u -m pytest tests/test_lmhead_gpu.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k 'lmhead or lora_proj or rowproj or projection'" \
  "k_rp:200:python tools/bench_rowproj.py" \
  "k_ab:500:python tools/step_ab.py 'MIFT_LM_NT=0' 'MIFT_LM_NT=1' 'MIFT_LM_NT=2' 'MIFT_LM_NT=3' 'MIFT_ROWPROJ_V=1'"
