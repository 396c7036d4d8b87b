#!/bin/bash
# round 6: half-layer pipeline units: GPU tests + sub-block cost calibration
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ab
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ab/tests:600:python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 240 --timeout-method thread -k 'half or graphs_match'" \
  "r6ab/cost27:300:python -u tools/half_layer_cost.py --model opt-2.7b --mb 12" \
  "r6ab/cost67:300:python -u tools/half_layer_cost.py --model opt-6.7b --mb 6"
