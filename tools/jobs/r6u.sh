#!/bin/bash
# round 6: what the dropout masks cost in the distilgpt2 step (diagnostic arms with other dropout rates)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6u
mkdir -p $O
bash tools/gpu_job.sh \
  "r6u/drop_ab:600:python -u tools/step_ab.py 'X=0' 'AB_MODEL_PDROP=0' 'AB_LORA_P=0' 'AB_MODEL_PDROP=0 AB_LORA_P=0' --blocks 6 --steps 20 --json $O/step_ab_dgpt_dropout_cost.json"
