#!/bin/bash
# round 5: folded-LN decode projections + host-side mask checks (decode target)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5m
mkdir -p $O
bash tools/gpu_job.sh \
  "r5m/tests:300:python -u -m pytest tests/test_kernels_gpu.py tests/test_infer_gpu.py -x -v --timeout 120 --timeout-method thread -k 'gemm_ln or infer or decode or generate or skinny'" \
  "r5m/probe:300:python -m mift.apps.gen_probe --repeat 5 && python -m mift.apps.gen_probe --repeat 5 --prompts distinct && MIFT_LN_FOLD=0 python -m mift.apps.gen_probe --repeat 5 && python -m mift.apps.gen_probe --repeat 5" \
  "r5m/kt:300:rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -m mift.apps.gen_probe --repeat 2 && python tools/gen_timeline.py $O/kt/run_kernel_trace.csv > $O/gen_timeline.txt"
