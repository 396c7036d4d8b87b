#!/bin/bash
# Round-3 second GPU pass: GPU tests (incl. pipeline stage graphs on one GPU over gloo, v2 attention),
# attention v1/v2 timings, PMC of the step, bench, OPT-2.7B PP4 rehearsal at real size.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
bash tools/gpu_job.sh \
  "b_tests:900:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "b_attn1:120:MIFT_ATTN_FWD=1 python tools/bench_attn.py" \
  "b_attn2:120:MIFT_ATTN_FWD=2 python tools/bench_attn.py" \
  "b_pmc:240:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc1 -o run -- python3 bench.py --steps 3 --warmup 1 --epoch_lines 0 && python tools/pmc_summary.py $O/pmc1 --top 40" \
  "b_bench:300:python bench.py" \
  "b_pp4:900:python tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 --seq 512 --mb 4 --accum 24 --steps 3"
