#!/bin/bash
# round 6: does rocprofv3 --pmc still abort on the graph-replayed OPT-2.7B step?
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6k
mkdir -p $O
P="python3 bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 12 --steps 1 --warmup 1 --epoch_lines 0"
timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES --output-format csv -d $O/o_waves -o run -- $P > $O/o_waves.log 2>&1
echo "rc=$?" >> $O/o_waves.log
