#!/bin/bash
# round 5: graph-branch concurrency evidence (kernel traces) + interleaved bench repeats
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5q
mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --epoch_lines 0"
bash tools/gpu_job.sh \
  "r5q/kt_q2:300:DEBUG_HIP_FORCE_GRAPH_QUEUES=2 rocprofv3 --kernel-trace --output-format csv -d $O/kt_q2 -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt_q2/run_kernel_trace.csv > $O/step_timeline_q2.txt" \
  "r5q/kt_np:300:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 rocprofv3 --kernel-trace --output-format csv -d $O/kt_np -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt_np/run_kernel_trace.csv > $O/step_timeline_np.txt" \
  "r5q/a1:200:$B" "r5q/b1:200:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B" "r5q/c1:200:DEBUG_HIP_FORCE_GRAPH_QUEUES=2 $B" \
  "r5q/a2:200:$B" "r5q/b2:200:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B" "r5q/c2:200:DEBUG_HIP_FORCE_GRAPH_QUEUES=2 $B" \
  "r5q/a3:200:$B" "r5q/b3:200:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B" "r5q/c3:200:DEBUG_HIP_FORCE_GRAPH_QUEUES=2 $B"
