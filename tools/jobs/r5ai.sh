#!/bin/bash
# round 5: proj_reduce with 4 columns per thread and batched slab loads (tests + kernel trace)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5ai
mkdir -p $O
bash tools/gpu_job.sh \
  "r5ai/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -v --timeout 120 --timeout-method thread -k 'proj or epilogue or opt or relu or skinny'" \
  "r5ai/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_proj_phase.py" \
  "r5ai/step_ab:300:python tools/step_ab.py 'MIFT_EPI_PROJ=1' --blocks 3 --steps 10 --json $O/step_dgpt.json"
