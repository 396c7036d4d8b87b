#!/bin/bash
# round 5: graph-branch concurrency with both HIP graph knobs (kernel trace for overlap) + repeats
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5w
mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --epoch_lines 0"
bash tools/gpu_job.sh \
  "r5w/kt:300:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt" \
  "r5w/a1:200:$B" "r5w/b1:200:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 $B" \
  "r5w/a2:200:$B" "r5w/b2:200:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 $B"
