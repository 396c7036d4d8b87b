#!/bin/bash
# round 5: 256-row 8-wave tiles (22: 256x96 3-stage, 23: 256x192, 24: 256x96 2-stage) vs the kept tiles on the
# distilgpt2 and OPT micro-batch GEMMs; OPT-2.7B dp1 mb48 with the epoch metric; OPT roofline (eager)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5g
mkdir -p $O
P="python3 bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 12 --steps 1 --warmup 1 --epoch_lines 0"
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
bash tools/gpu_job.sh \
  "r5g/tiles_dgpt:400:TILES=0,7,9,22,23,24 python tools/bench_kernels.py --only dgpt --json $O/tiles_dgpt.json" \
  "r5g/tiles_opt:500:TILES=0,7,8,22,23,24 python tools/bench_kernels.py --only optm_pp --json $O/tiles_opt.json" \
  "r5g/opt_dp1_mb48:900:python bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 5 --warmup 2" \
  "r5g/o_sq:300:MIFT_GRAPH=off timeout -s KILL 280 rocprofv3 --pmc $SQ --output-format csv -d $O/o_sq -o run -- $P" \
  "r5g/o_fetch:300:MIFT_GRAPH=off timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/o_fetch -o run -- $P" \
  "r5g/o_write:300:MIFT_GRAPH=off timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/o_write -o run -- $P" \
  "r5g/o_sum:60:python tools/pmc_summary.py $O/o_sq $O/o_fetch $O/o_write --top 40"
