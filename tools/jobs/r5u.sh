#!/bin/bash
# round 5: fc1's dT from the fc2-dgrad epilogue (OPT) — tests + OPT step A/B
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5u
mkdir -p $O
bash tools/gpu_job.sh \
  "r5u/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_graph_gpu.py -x -v --timeout 120 --timeout-method thread -k 'projection or fused or opt or graph'" \
  "r5u/step_ab_opt:400:python tools/step_ab.py --model facebook/opt-2.7b 'MIFT_EPI_DT=1' 'MIFT_EPI_DT=0' --blocks 4 --steps 5 --json $O/step_ab_opt_epi_dt.json"
