#!/bin/bash
# round 6: 4-wave 256x256 GEMM (tile 10) numerics vs tile 8, timing vs tile 8 / hipBLASLt; baseline bench
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 180 python -u tools/bench_gemm4.py --check-only > $O/check.log 2>&1 && \
timeout -k 10 400 python -u tools/bench_gemm4.py --json $O/bench_gemm4.json > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench_dgpt.log 2>&1
