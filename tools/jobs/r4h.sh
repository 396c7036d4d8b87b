#!/bin/bash
# round 4: skinny decode GEMM + fused decode tail; lse / optimizer arrival counters already in
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4h
mkdir -p $O
bash tools/gpu_job.sh \
  "r4h/tests:500:python -u -m pytest tests/test_kernels_gpu.py tests/test_infer_gpu.py -k 'skinny or decode or splitk or projection or infer or generate or padded or graphed' -x -q --timeout 120 --timeout-method thread" \
  "r4h/gen_eager:200:MIFT_GEN_GRAPH=0 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4h/gen_graph:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4h/gen_graph_distinct:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5 --prompts distinct" \
  "r4h/gen_graph_noskinny:200:MIFT_GEMM_SKINNY=0 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4h/kt_decode:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktdec -o run -- python3 scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 3"
