#!/bin/bash
# round 5: hipBLASLt kernel names / times for the OPT layer GEMMs (kernel trace)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}/tools
O=../gpurun_out/r5am
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 blas_kernel_names.py > $O/run.log 2>&1
