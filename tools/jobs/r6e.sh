#!/bin/bash
# round 6: GEMM GPU tests (tile 10 bit-identity + every tile), OPT step A/B (tile 10 auto vs forced 8), benches
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6e
mkdir -p $O
bash tools/gpu_job.sh \
  "r6e/tests:600:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'gemm or relu or nontemporal or projection'" \
  "r6e/opt_ab:600:python -u tools/step_ab.py 'MIFT_GEMM_T10=0' 'MIFT_X=1' --model opt-2.7b --blocks 4 --steps 3 --json $O/step_ab_opt_t10.json" \
  "r6e/opt_mb48:900:python bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 5 --warmup 2 --epoch_lines 0" \
  "r6e/dgpt:300:python bench.py"
