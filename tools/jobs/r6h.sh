#!/bin/bash
# round 6: one-launch q/k/v multi-adapter pack: tests + OPT step kernel census
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6h
mkdir -p $O
bash tools/gpu_job.sh \
  "r6h/tests:900:python -u -m pytest tests/test_fused_gpu.py tests/test_graph_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread" \
  "r6h/kt_opt:600:rocprofv3 --kernel-trace --output-format csv -d $O/kto -o run -- python3 bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 3 --warmup 2 --epoch_lines 0"
