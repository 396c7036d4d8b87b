#!/bin/bash
# round 6: minimal repro — N-kernel torch graph replayed under rocprofv3 --pmc (packet capture on)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6m
mkdir -p $O
for N in 64 512; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES --output-format csv -d $O/n$N -o run -- python3 tools/diag_pmc_graph.py $N 2 > $O/n$N.log 2>&1
  rc=$?; echo "rc=$rc" >> $O/n$N.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES --output-format csv -d $O/n4096 -o run -- python3 tools/diag_pmc_graph.py 4096 2 > $O/n4096.log 2>&1
echo "rc=$?" >> $O/n4096.log
