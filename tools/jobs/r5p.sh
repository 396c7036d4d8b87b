#!/bin/bash
# round 5: do parallel graph branches (the side-stream LoRA weight gradients) run concurrently?
# HIP runtime graph knobs, one process each (read at runtime init)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5p
mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --epoch_lines 0"
bash tools/gpu_job.sh \
  "r5p/base1:200:$B" \
  "r5p/nopkt1:200:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B" \
  "r5p/q2:200:DEBUG_HIP_FORCE_GRAPH_QUEUES=2 $B" \
  "r5p/nopkt_q2:200:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 $B" \
  "r5p/base2:200:$B" \
  "r5p/nopkt2:200:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B"
