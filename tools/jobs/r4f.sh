#!/bin/bash
# round 4: write-through (sc1) last-block hand-off in opt_stats / lmhead_lse — tests, bench, step timeline
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4f
mkdir -p $O
bash tools/gpu_job.sh \
  "r4f/tests:400:python -u -m pytest tests/test_optimizer_fold_gpu.py tests/test_lmhead_gpu.py tests/test_graph_gpu.py tests/test_loss_scale_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "r4f/bench:300:python bench.py --steps 20 --warmup 5" \
  "r4f/kt_step:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv"
