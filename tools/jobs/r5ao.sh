#!/bin/bash
# round 5: non-temporal C stores by output size (default) vs off / all, OPT mb48; NT store test
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5ao
mkdir -p $O
bash tools/gpu_job.sh \
  "r5ao/tests:300:python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k 'nontemporal or relu or epilogue'" \
  "r5ao/step_opt:600:python tools/step_ab.py --model facebook/opt-2.7b 'MIFT_EPI_NT=0' 'MIFT_EPI_NT=1' 'MIFT_NT_DEFAULT=1' --blocks 4 --steps 5 --mb 48 --json $O/step_ab_opt_nt_auto.json"
