#!/bin/bash
# round 5: MODE 2 row projection at K=7680 (OPT q/k/v dT) — numerics + timing against lora_proj's own kernel
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5z
mkdir -p $O

timeout -k 10 300 python -u tools/bench_rowproj_opt.py --json $O/bench_rowproj_opt.json > $O/bench.log 2>&1
