#!/bin/bash
# Round-3 eleventh GPU pass: lora_proj routing tests, attention batch sweep (per-CU balance), cost of
# the deterministic slab reductions.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "l_tests:200:python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k 'lora_proj or rowproj'" \
  "l_sweep:200:python tools/bench_attn.py --sweep" \
  "l_ab:400:python tools/step_ab.py 'MIFT_DETERMINISTIC=1' 'MIFT_DETERMINISTIC=0'"
