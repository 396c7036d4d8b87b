#!/bin/bash
# round 5: non-temporal GEMM C stores (A/B): OPT 4-block step at mb48 and the distilgpt2 step
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5an
mkdir -p $O
bash tools/gpu_job.sh \
  "r5an/step_opt:500:python tools/step_ab.py --model facebook/opt-2.7b 'MIFT_EPI_NT=0' 'MIFT_EPI_NT=1' --blocks 4 --steps 5 --mb 48 --json $O/step_ab_opt_nt.json" \
  "r5an/step_dgpt:300:python tools/step_ab.py 'MIFT_EPI_NT=0' 'MIFT_EPI_NT=1' --blocks 6 --steps 10 --json $O/step_ab_dgpt_nt.json"
