#!/bin/bash
# round 4: skinny-GEMM epilogue-operand prefetch (MIFT_SKINNY_PF) — tests, per-op A/B, graphed decode A/B
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4u
mkdir -p $O
bash tools/gpu_job.sh \
  "r4u/tests:300:python -u -m pytest tests/test_kernels_gpu.py tests/test_infer_gpu.py -k 'skinny or gemm_ln or decode or splitk or projection or generate or graphed' -x -q --timeout 120 --timeout-method thread" \
  "r4u/ops:300:python tools/bench_decode.py --json $O/ops.json" \
  "r4u/g1a:200:MIFT_SKINNY_PF=1 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4u/g0a:200:MIFT_SKINNY_PF=0 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4u/g1b:200:MIFT_SKINNY_PF=1 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4u/g0b:200:MIFT_SKINNY_PF=0 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5"
