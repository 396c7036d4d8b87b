#!/bin/bash
# round 6: LM-head forward E stores non-temporal (MIFT_LM_DBG bit 4, A/B) in the persistent kernel
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6aj
mkdir -p $O
bash tools/gpu_job.sh \
  "r6aj/ab:600:python -u tools/step_ab.py 'MIFT_LM_DBG=0' 'MIFT_LM_DBG=16' --blocks 6 --steps 20 --json $O/step_ab_dgpt_lm_e_nt.json"
