#!/bin/bash
# round 5: persistent fused LM-head forward v2 + attention: transposed-output P·V (MIFT_ATTN_OT) and
# XCD-aware tile mapping (MIFT_ATTN_XCD) — GPU tests, A/Bs, whole step
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5e
mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --epoch_lines 0"
bash tools/gpu_job.sh \
  "r5e/test_lm:500:python -u -m pytest tests/test_lmhead_gpu.py tests/test_graph_gpu.py tests/test_fused_gpu.py tests/test_kernels_gpu.py tests/test_infer_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "r5e/bench_lm:300:python tools/bench_lm_persist.py" \
  "r5e/attn_ot:300:python tools/bench_attn.py --ab MIFT_ATTN_OT=0,1" \
  "r5e/attn_xcd:300:python tools/bench_attn.py --ab MIFT_ATTN_XCD=0,1 --only opt-2.7b,opt-6.7b" \
  "r5e/on1:200:$B" \
  "r5e/off1:200:MIFT_LM_PERSIST=0 MIFT_LM_GROUP=0 MIFT_ATTN_OT=0 $B" \
  "r5e/on2:200:$B" \
  "r5e/off2:200:MIFT_LM_PERSIST=0 MIFT_LM_GROUP=0 MIFT_ATTN_OT=0 $B" \
  "r5e/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt"
