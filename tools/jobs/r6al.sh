#!/bin/bash
# round 6: BASELINE configs 3 (OPT-2.7B PP4 x V4, mb 12 x 8) and 4 (2dp x 4pp) with half-layer stage boundaries, rehearsed
# at real size on one GPU against the same-DP run without pipelining
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6al
mkdir -p $O
(while sleep 45; do echo "heartbeat $(date +%T)" >> $O/heartbeat.txt; done) &
HB=$!
bash tools/gpu_job.sh \
  "r6al/c3:600:python -u tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 --virtual 4 --mb 12 --accum 8 --steps 3 --partition halves --timeout 500 > $O/rehearse_config3_opt27b_pp4v4_halves.json" \
  "r6al/c4:600:python -u tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 --dp 2 --mb 12 --accum 8 --steps 3 --partition halves --timeout 500 > $O/rehearse_config4_opt27b_dp2pp4_halves.json"
RC=$?
kill $HB
exit $RC
