#!/bin/bash
# round 6: LoRA K-extension operands staged into LDS during the last k-tile (NSTAGE >= 2 tiles): tests, stamps, step A/B
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6au
mkdir -p $O
bash tools/gpu_job.sh \
  "r6au/tests:600:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread -k 'gemm or lora or ext or epilogue or fused'" \
  "r6au/stamps:300:python -u tools/gemm_stamps.py --shapes dgpt --tiles 9,7 --ext" \
  "r6au/ab:600:python -u tools/step_ab.py 'MIFT_EXT_LDS=0' 'MIFT_EXT_LDS=1' --blocks 8 --steps 20 --json $O/step_ab_dgpt_ext_lds.json"
