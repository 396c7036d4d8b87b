#!/bin/bash
# round 6: in-step sweep of the LM-head forward raster group (default 4 at K = 768)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6am
mkdir -p $O
bash tools/gpu_job.sh \
  "r6am/ab:600:python -u tools/step_ab.py 'MIFT_LM_GROUP=4' 'MIFT_LM_GROUP=2' 'MIFT_LM_GROUP=3' 'MIFT_LM_GROUP=1' --blocks 8 --steps 20 --json $O/step_ab_dgpt_lm_group2.json"
