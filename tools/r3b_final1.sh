#!/bin/bash
# Round-3 (session 2) evidence, part 1: GPU tests, smoke, driver-style bench, kernel trace + PMC of the step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r3bf
mkdir -p $O
bash tools/gpu_job.sh \
  "f_tests:500:python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread" \
  "f_smoke:150:python __graft_entry__.py smoke" \
  "f_bench:200:python bench.py" \
  "f_kt:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0" \
  "f_pmc:150:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 3 --warmup 1 --epoch_lines 0"
