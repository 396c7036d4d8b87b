#!/bin/bash
# round 5: where the GEMM projection phase's time goes (OPT fc1 shape), kernel trace
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5ah
mkdir -p $O
bash tools/gpu_job.sh \
  "r5ah/bench:300:python -u tools/bench_proj_phase.py" \
  "r5ah/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_proj_phase.py"
