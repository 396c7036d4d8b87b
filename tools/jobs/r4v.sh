#!/bin/bash
# round 4: 8-wave 128-row tiles (tiles 20 / 21) — correctness, distilgpt2 and OPT micro-batch sweeps
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4v
mkdir -p $O
bash tools/gpu_job.sh \
  "r4v/tests:300:python -u -m pytest tests/test_kernels_gpu.py -k 'splitk_tail_fused or epilogue_projection' -x -q --timeout 120 --timeout-method thread" \
  "r4v/dgpt:300:TILES=0,3,7,9,20,21 python tools/bench_kernels.py --only dgpt --json $O/dgpt.json" \
  "r4v/optm:400:TILES=0,3,7,20,21 python tools/bench_kernels.py --only optm_small --json $O/optm.json"
