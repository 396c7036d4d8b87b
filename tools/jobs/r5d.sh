#!/bin/bash
# round 5: persistent fused LM-head forward v2 (labels by LDS-DMA, next tile's A issued before the
# epilogue, K-based raster group) — GPU LM-head + graph tests, A/B, whole step on/off interleaved
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5d
mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --epoch_lines 0"
bash tools/gpu_job.sh \
  "r5d/test_lm:400:python -u -m pytest tests/test_lmhead_gpu.py tests/test_graph_gpu.py tests/test_fused_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "r5d/bench_lm:300:python tools/bench_lm_persist.py" \
  "r5d/on1:200:$B" \
  "r5d/off1:200:MIFT_LM_PERSIST=0 MIFT_LM_GROUP=0 $B" \
  "r5d/on2:200:$B" \
  "r5d/off2:200:MIFT_LM_PERSIST=0 MIFT_LM_GROUP=0 $B" \
  "r5d/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt"
