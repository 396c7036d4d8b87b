#!/bin/bash
# Round-3 seventh GPU pass: eager DDP double-count fix (diag + tests), side-stream wgrad A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "h_ddp:300:python tools/diag_ddp_eager.py --graph 0 --steps 3" \
  "h_tests:400:python -u -m pytest tests/test_pipeline_gpu.py tests/test_fused_gpu.py -q --timeout 300 --timeout-method thread" \
  "h_ab:400:python tools/step_ab.py 'MIFT_GRAPH_SIDE=0' 'MIFT_GRAPH_SIDE=1'"
