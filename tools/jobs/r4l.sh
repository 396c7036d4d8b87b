#!/bin/bash
# round 4: batched LN-prologue loads, long-K / wide-N decode GEMMs back on tiles; per-op decode timings
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4l
mkdir -p $O
bash tools/gpu_job.sh \
  "r4l/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_infer_gpu.py -k 'skinny or decode or infer or generate or padded or graphed or gemm_ln' -x -q --timeout 120 --timeout-method thread" \
  "r4l/bench_decode:200:python tools/bench_decode.py --json $O/bench_decode.json" \
  "r4l/gen_graph:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4l/gen_graph_distinct:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5 --prompts distinct" \
  "r4l/kt_decode:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktdec -o run -- python3 scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 3"
