#!/bin/bash
# Round-3 13th GPU pass: in-kernel wgrad slab reduction (tests, step A/B), attention split tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "n_tests:300:python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k 'wgrad or attention or flash or lora'" \
  "n_ab:400:python tools/step_ab.py 'MIFT_WGRAD_FIN=1' 'MIFT_WGRAD_FIN=0'"
