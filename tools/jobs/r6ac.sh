#!/bin/bash
# round 6: one-rank stage times of BASELINE configs 3 / 5 with half-layer vs whole-layer partitions
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ac
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ac/c3h:900:python -u tools/stage_time.py --config 3 --partition halves --json $O/stage_time_config3_halves.json" \
  "r6ac/c3b:900:python -u tools/stage_time.py --config 3 --partition balanced --json $O/stage_time_config3_balanced.json"
