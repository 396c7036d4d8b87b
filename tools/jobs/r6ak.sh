#!/bin/bash
# round 6: BASELINE config 5 (OPT-6.7B PP8 x V2, mb 6 x 16) with half-layer stage boundaries, rehearsed at real size on
# one GPU (8 rank processes, gloo transport, production engine + stage graphs) against the dp1 run of the same data
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ak
mkdir -p $O
(while sleep 45; do echo "heartbeat $(date +%T)" >> $O/heartbeat.txt; done) &
HB=$!
bash tools/gpu_job.sh \
  "r6ak/c5:1000:python -u tools/rehearse_pp.py --model facebook/opt-6.7b --pp 8 --virtual 2 --mb 6 --accum 16 --steps 3 --partition halves --timeout 900 > $O/rehearse_opt67b_pp8v2_halves.json"
RC=$?
kill $HB
exit $RC
