#!/bin/bash
# round 4: decode_tail block-size A/B (kernel durations from a trace of the per-op bench)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4m
mkdir -p $O
bash tools/gpu_job.sh \
  "r4m/tests:300:python -u -m pytest tests/test_kernels_gpu.py tests/test_infer_gpu.py -k 'decode or gemm_ln or graphed' -x -q --timeout 120 --timeout-method thread" \
  "r4m/kt_bench_decode:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_decode.py --json $O/bench_decode.json"
