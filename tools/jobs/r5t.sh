#!/bin/bash
# round 5 checkpoint: full GPU suite, smoke, bench x2, step kernel trace, decode probe
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5t
mkdir -p $O
bash tools/gpu_job.sh \
  "r5t/gpu_tests:1000:python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread" \
  "r5t/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r5t/bench1:300:python bench.py" \
  "r5t/bench2:300:python bench.py" \
  "r5t/probe:200:python -m mift.apps.gen_probe --repeat 5 && python -m mift.apps.gen_probe --repeat 5 --prompts distinct" \
  "r5t/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt"
