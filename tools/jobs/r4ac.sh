#!/bin/bash
# round 4: LM-head dgrad in-launch reduction (MIFT_LM_FIN) — tests, head bench A/B, step bench A/B
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4ac
mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --epoch_lines 0"
bash tools/gpu_job.sh \
  "r4ac/tests:300:python -u -m pytest tests/test_lmhead_gpu.py tests/test_graph_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "r4ac/head1:200:python tools/bench_lmhead.py" \
  "r4ac/head0:200:MIFT_LM_FIN=0 python tools/bench_lmhead.py" \
  "r4ac/on1:200:$B" \
  "r4ac/off1:200:MIFT_LM_FIN=0 $B" \
  "r4ac/on2:200:$B" \
  "r4ac/off2:200:MIFT_LM_FIN=0 $B" \
  "r4ac/on3:200:$B" \
  "r4ac/off3:200:MIFT_LM_FIN=0 $B"
