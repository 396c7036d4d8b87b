#!/bin/bash
# round 5: 256x256 epilogue: LDS-only barrier before the projection phase, grouped operand requests (A/B) + affected tests
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5af
mkdir -p $O
bash tools/gpu_job.sh \
  "r5af/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -v --timeout 120 --timeout-method thread -k 'relu or epilogue or opt or proj'" \
  "r5af/epi:400:python -u tools/bench_opt_epilogue.py --json $O/bench_opt_epilogue.json"
bash tools/gpu_job.sh \
  "r5af/step_ab:500:python tools/step_ab.py --model facebook/opt-2.7b 'MIFT_EPI_PFG=0 MIFT_EPI_SYNC=1' 'MIFT_EPI_PFG=1' --blocks 4 --steps 5 --mb 48 --json $O/step_ab_opt_epi_pfg.json"
