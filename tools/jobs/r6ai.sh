#!/bin/bash
# round 6: 4-wave loop with counted LDS waits (no lgkmcnt(0) drains right after reads): bit identity, GEMM bench, OPT step A/B
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ai
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ai/tests:600:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'gemm or 4wave or hoisted'" \
  "r6ai/bench:600:python -u tools/bench_gemm4.py --json $O/bench_gemm4_counted_lgkm.json" \
  "r6ai/opt_ab:600:python -u tools/step_ab.py 'MIFT_GEMM_T10=0' 'MIFT_X=1' --model opt-2.7b --blocks 4 --steps 3 --json $O/step_ab_opt_t10_counted.json"
