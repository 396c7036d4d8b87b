#!/bin/bash
# round 6: staged epilogue on every tile: bit-identity tests, step A/B (distilgpt2, OPT mb12), benches
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6f
mkdir -p $O
bash tools/gpu_job.sh \
  "r6f/tests:900:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'gemm or relu or nontemporal or projection'" \
  "r6f/dgpt_ab:600:python -u tools/step_ab.py 'MIFT_EPI_STAGED=0' 'MIFT_EPI_STAGED=1' --blocks 6 --steps 20 --json $O/step_ab_dgpt_staged.json" \
  "r6f/opt_ab:600:python -u tools/step_ab.py 'MIFT_EPI_STAGED=0' 'MIFT_EPI_STAGED=1' --model opt-2.7b --blocks 4 --steps 3 --json $O/step_ab_opt_staged.json" \
  "r6f/dgpt:300:python bench.py"
