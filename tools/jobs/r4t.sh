#!/bin/bash
# round 4: half-depth (KB = 32) GEMM rings — correctness, then the distilgpt2 tile sweep
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4t
mkdir -p $O
bash tools/gpu_job.sh \
  "r4t/tests:300:python -u -m pytest tests/test_kernels_gpu.py -k 'half_depth or splitk_tail_fused or epilogue_projection' -x -q --timeout 120 --timeout-method thread" \
  "r4t/dgpt1:300:TILES=0,7,9,16,17,18,19 python tools/bench_kernels.py --only dgpt --json $O/dgpt1.json" \
  "r4t/dgpt2:300:TILES=0,7,9,16,17,18,19 python tools/bench_kernels.py --only dgpt --json $O/dgpt2.json"
