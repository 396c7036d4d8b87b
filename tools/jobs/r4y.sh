#!/bin/bash
# round 4: HIP graph execution knobs — does the side-stream wgrad branch run concurrently in the replayed step?
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4y
mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --epoch_lines 0"
bash tools/gpu_job.sh \
  "r4y/def1:200:$B" \
  "r4y/q2:200:DEBUG_HIP_FORCE_GRAPH_QUEUES=2 $B" \
  "r4y/q4:200:DEBUG_HIP_FORCE_GRAPH_QUEUES=4 $B" \
  "r4y/pc0:200:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B" \
  "r4y/pc1:200:DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 $B" \
  "r4y/def2:200:$B" \
  "r4y/q4b:200:DEBUG_HIP_FORCE_GRAPH_QUEUES=4 $B" \
  "r4y/side0:200:MIFT_SIDE_STREAM=0 $B"
