#!/bin/bash
# round 6: hoisted dropout hashes in the GEMM epilogues: bit identity + step A/B
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6p
mkdir -p $O
bash tools/gpu_job.sh \
  "r6p/tests:600:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'hoisted or 4wave'" \
  "r6p/dgpt_ab:600:python -u tools/step_ab.py 'MIFT_EPI_HOIST=0' 'MIFT_EPI_HOIST=1' --blocks 6 --steps 20 --json $O/step_ab_dgpt_hoist.json" \
  "r6p/opt_ab:600:python -u tools/step_ab.py 'MIFT_EPI_HOIST=0' 'MIFT_EPI_HOIST=1' 'MIFT_EPI_HOIST=1 MIFT_GEMM_T10=1' --model opt-2.7b --blocks 4 --steps 3 --json $O/step_ab_opt_hoist.json"
