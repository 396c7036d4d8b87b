#!/bin/bash
# round 6: per-block stamps of tiles 8 / 10 (prologue / loop / epilogue split)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 200 python -u tools/gemm_stamps.py > $O/stamps.log 2>&1
