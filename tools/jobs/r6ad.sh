#!/bin/bash
# round 6: one-rank stage times of BASELINE config 5 (OPT-6.7B PP8) with half-layer vs whole-layer partitions
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ad
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ad/c5h:1000:python -u tools/stage_time.py --config 5 --partition halves --json $O/stage_time_config5_halves.json" \
  "r6ad/c5b:1000:python -u tools/stage_time.py --config 5 --partition balanced --json $O/stage_time_config5_balanced.json"
