#!/bin/bash
# Round-3 eighth GPU pass: 16-B LayerNorm kernels (tests, step A/B), OPT ReLU-kink diagnostic.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "i_ln_tests:300:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -q --timeout 120 --timeout-method thread -k 'layer_norm or rowproj or gpt2 or opt'" \
  "i_relu:200:python tools/diag_opt_relu.py" \
  "i_ab:400:python tools/step_ab.py 'MIFT_LN_V=0' 'MIFT_LN_V=1'"
