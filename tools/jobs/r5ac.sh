#!/bin/bash
# round 5: epilogue cost of the OPT-2.7B block GEMMs at micro-batch 48 (phased 256x256 tile)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5ac
mkdir -p $O
timeout -k 10 400 python -u tools/bench_opt_epilogue.py --json $O/bench_opt_epilogue.json > $O/bench.log 2>&1
