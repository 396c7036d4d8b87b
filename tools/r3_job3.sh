#!/bin/bash
# Round-3 third GPU pass: PP graph fix (per-slot pools) + eager-vs-graph diagnostics + PP4 rehearsal
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
bash tools/gpu_job.sh \
  "c_diag:300:python tools/diag_graph_eager.py --model facebook/opt-125m --precision fp16 --steps 3" \
  "c_tests:600:python -u -m pytest tests/test_pipeline_gpu.py tests/test_graph_gpu.py tests/test_kernels_gpu.py -q --timeout 300 --timeout-method thread -k 'pipeline or graph or attention_fwd_v2 or whole_sequence'" \
  "c_pp4:900:python tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 --seq 512 --mb 4 --accum 24 --steps 3"
