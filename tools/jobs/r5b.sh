#!/bin/bash
# round 5: roofline evidence — SQ / FETCH_SIZE / WRITE_SIZE passes (one counter group per run) on the
# replayed distilgpt2 step and on OPT-2.7B dp1 micro-batch 12 (fp16, seq 512)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5b
mkdir -p $O
D="python3 bench.py --steps 3 --warmup 1 --epoch_lines 0"
P="python3 bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 12 --steps 1 --warmup 1 --epoch_lines 0"
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
bash tools/gpu_job.sh \
  "r5b/d_sq:200:timeout -s KILL 180 rocprofv3 --pmc $SQ --output-format csv -d $O/d_sq -o run -- $D" \
  "r5b/d_fetch:200:timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/d_fetch -o run -- $D" \
  "r5b/d_write:200:timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/d_write -o run -- $D" \
  "r5b/d_sum:60:python tools/pmc_summary.py $O/d_sq $O/d_fetch $O/d_write --top 40" \
  "r5b/o_sq:300:timeout -s KILL 280 rocprofv3 --pmc $SQ --output-format csv -d $O/o_sq -o run -- $P" \
  "r5b/o_fetch:300:timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/o_fetch -o run -- $P" \
  "r5b/o_write:300:timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/o_write -o run -- $P" \
  "r5b/o_sum:60:python tools/pmc_summary.py $O/o_sq $O/o_fetch $O/o_write --top 40"
