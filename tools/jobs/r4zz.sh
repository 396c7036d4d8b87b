#!/bin/bash
# round 4 closing evidence (second pass, after the dK/dV occupancy, tile-rule, prefetch and LN-handoff changes): GPU suite, smoke, bench, step kernel trace + PMC, decode, attention
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4zz
mkdir -p $O
bash tools/gpu_job.sh \
  "r4zz/pytest:900:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r4zz/smoke:200:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "r4zz/bench:300:python bench.py --steps 20 --warmup 5" \
  "r4zz/kt_step:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv" \
  "r4zz/pmc_step:240:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 3 --warmup 1 --epoch_lines 0 && python tools/pmc_summary.py $O/pmc --top 30" \
  "r4zz/gen_graph:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4zz/gen_graph_distinct:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5 --prompts distinct" \
  "r4zz/bench_attn:200:python tools/bench_attn.py --json $O/bench_attn.json"
