#!/bin/bash
# round 4: one-wave 128x96 auto rule — GEMM tests, OPT micro-batch shapes (auto), OPT-2.7B dp1 mb 2/4/8 steps
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4x
mkdir -p $O
bash tools/gpu_job.sh \
  "r4x/tests:300:python -u -m pytest tests/test_kernels_gpu.py -k 'splitk_tail_fused or epilogue_projection or half_depth' -x -q --timeout 120 --timeout-method thread" \
  "r4x/optpp:300:TILES=0,7 python tools/bench_kernels.py --only optm_pp --json $O/optpp.json" \
  "r4x/mb:600:python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 2,4,8 --steps 3 --warmup 2 --out $O/mb.jsonl"
