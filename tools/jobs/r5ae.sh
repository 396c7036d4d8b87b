#!/bin/bash
# round 5: sign-bits tests (fixed reference tile) + the rest of the affected GPU tests
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5ae
mkdir -p $O
bash tools/gpu_job.sh \
  "r5ae/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_pipeline_gpu.py -v --timeout 120 --timeout-method thread -k 'relu or epilogue or opt or proj or gemm'"
