#!/bin/bash
# round 4: two-level arrival counters (lmhead_lse / opt_stats), small-grid split-K for decode GEMMs
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4g
mkdir -p $O
bash tools/gpu_job.sh \
  "r4g/tests:500:python -u -m pytest tests/test_optimizer_fold_gpu.py tests/test_lmhead_gpu.py tests/test_infer_gpu.py tests/test_graph_gpu.py tests/test_kernels_gpu.py -k 'fold or lmhead or splitk or projection or infer or decode or graph or adamw or generate or padded' -x -q --timeout 120 --timeout-method thread" \
  "r4g/bench:300:python bench.py --steps 20 --warmup 5" \
  "r4g/kt_step:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv" \
  "r4g/gen_eager:200:MIFT_GEN_GRAPH=0 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4g/gen_graph:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4g/kt_decode:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktdec -o run -- python3 scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 3"
