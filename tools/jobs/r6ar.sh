#!/bin/bash
# round 6: cross-lane reductions at distance 16 / 32 through v_permlane16/32_swap (attention, LM head, row passes)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6ar
mkdir -p $O
bash tools/gpu_job.sh \
  "r6ar/gpu_tests:1000:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r6ar/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt" \
  "r6ar/bench:300:python -u bench.py --steps 20 --warmup 5 --epoch_lines 0 > $O/bench.jsonl && python -u bench.py --steps 20 --warmup 5 --epoch_lines 0 >> $O/bench.jsonl"
