#!/bin/bash
# round 5: pipeline evidence — interleaved stage-graph GPU tests, per-rank isolated stage times of BASELINE
# configs 3/4 (OPT-2.7B PP4) and 5 (OPT-6.7B PP8), OPT-2.7B dp1 with the epoch metric, OPT roofline passes
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5f
mkdir -p $O
P="python3 bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 12 --steps 1 --warmup 1 --epoch_lines 0"
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
bash tools/gpu_job.sh \
  "r5f/test_pp:600:python -u -m pytest tests/test_pipeline_gpu.py -x -v --timeout 240 --timeout-method thread" \
  "r5f/stage3:600:python tools/stage_time.py --config 3 --json $O/stage_time_config3.json" \
  "r5f/stage5:900:python tools/stage_time.py --config 5 --json $O/stage_time_config5.json" \
  "r5f/opt_dp1_mb48:600:python bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 48 --steps 5 --warmup 2" \
  "r5f/o_sq:300:MIFT_GRAPH=off timeout -s KILL 280 rocprofv3 --pmc $SQ --output-format csv -d $O/o_sq -o run -- $P" \
  "r5f/o_fetch:300:MIFT_GRAPH=off timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/o_fetch -o run -- $P" \
  "r5f/o_write:300:MIFT_GRAPH=off timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/o_write -o run -- $P" \
  "r5f/o_sum:60:python tools/pmc_summary.py $O/o_sq $O/o_fetch $O/o_write --top 40"
