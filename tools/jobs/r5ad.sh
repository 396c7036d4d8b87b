#!/bin/bash
# round 5: ReLU sign bits for OPT's fc2-dgrad epilogue + hoisted projection-phase weights
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5ad
mkdir -p $O
bash tools/gpu_job.sh \
  "r5ad/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -v --timeout 120 --timeout-method thread -k 'relu or epilogue or opt or proj'" \
  "r5ad/epi:400:python -u tools/bench_opt_epilogue.py --json $O/bench_opt_epilogue.json" \
  "r5ad/step_ab:500:python tools/step_ab.py --model facebook/opt-2.7b 'MIFT_RELU_BITS=0' 'MIFT_RELU_BITS=1' --blocks 4 --steps 5 --mb 48 --json $O/step_ab_opt_relu_bits.json"
