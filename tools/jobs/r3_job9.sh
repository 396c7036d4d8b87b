#!/bin/bash
# Round-3 ninth GPU pass: epilogue LoRA projection (tests + step A/B) and the whole GPU suite.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "j_proj:200:python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k 'projection'" \
  "j_ab:400:python tools/step_ab.py 'MIFT_EPI_PROJ=1' 'MIFT_EPI_PROJ=0'" \
  "j_all:900:python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread"
