#!/bin/bash
# round 6: tile 10 with the lean / staged epilogue: numerics, stamps, plain + training-epilogue timing
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 180 python -u tools/bench_gemm4.py --check-only > $O/check.log 2>&1 && \
timeout -k 10 200 python -u tools/gemm_stamps.py > $O/stamps.log 2>&1 && \
timeout -k 10 400 python -u tools/bench_gemm4.py --json $O/bench_gemm4.json > $O/bench.log 2>&1 && \
TILES=8,10 timeout -k 10 400 python -u tools/bench_kernels.py --only optm --json $O/optm.json > $O/optm.log 2>&1
