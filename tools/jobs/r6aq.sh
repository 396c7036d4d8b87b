#!/bin/bash
# round 6 final-candidate evidence: full GPU suite, smoke, bench x2, decode probe, step kernel trace, OPT-2.7B dp1 mb48
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6aq
mkdir -p $O
bash tools/gpu_job.sh \
  "r6aq/gpu_tests:1000:python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread" \
  "r6aq/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6aq/bench1:300:python bench.py > $O/bench.jsonl" \
  "r6aq/bench2:300:python bench.py >> $O/bench.jsonl" \
  "r6aq/probe:200:python -m mift.apps.gen_probe --repeat 10 && python -m mift.apps.gen_probe --repeat 10 --prompts distinct > $O/gen_probe.txt 2>&1" \
  "r6aq/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt" \
  "r6aq/opt_mb48:900:python bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 5 --warmup 2 > $O/opt_mb48.jsonl"
