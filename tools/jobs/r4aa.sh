#!/bin/bash
# round 4: LN backward + residual-dropout backward + dT in one pass (GradHandoff) — tests, bench A/B, trace
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4aa
mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --epoch_lines 0"
bash tools/gpu_job.sh \
  "r4aa/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_graph_gpu.py -k 'ln_bwd_mask_proj or handoff or fused or graph or rowproj or mask_proj or layer_norm' -x -q --timeout 120 --timeout-method thread" \
  "r4aa/on1:200:$B" \
  "r4aa/off1:200:MIFT_LN_MASK_PROJ=0 $B" \
  "r4aa/on2:200:$B" \
  "r4aa/off2:200:MIFT_LN_MASK_PROJ=0 $B" \
  "r4aa/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv"
