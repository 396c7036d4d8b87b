#!/bin/bash
# round 5: column split of the wide distilgpt2 GEMMs (phased 256x256 on 2048 columns + a second tile)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5aa
mkdir -p $O
timeout -k 10 300 python -u tools/bench_split_n.py --json $O/bench_split_n.json > $O/bench.log 2>&1
