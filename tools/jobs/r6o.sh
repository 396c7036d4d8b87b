#!/bin/bash
# round 6: roofline counter passes on the GRAPH-REPLAYED OPT-2.7B mb12 step (HIP graph packet capture off:
# with it on, rocprofv3 --pmc crashes inside hipGraphLaunch, r6k) and on the replayed distilgpt2 step
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6o
mkdir -p $O
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
D="python3 bench.py --steps 3 --warmup 1 --epoch_lines 0"
P="python3 bench.py --model facebook/opt-2.7b --pp 1 --micro_batch 12 --steps 1 --warmup 1 --epoch_lines 0"
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
bash tools/gpu_job.sh \
  "r6o/o_sq:300:timeout -s KILL 280 rocprofv3 --pmc $SQ --output-format csv -d $O/o_sq -o run -- $P" \
  "r6o/o_fetch:300:timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/o_fetch -o run -- $P" \
  "r6o/o_write:300:timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/o_write -o run -- $P" \
  "r6o/o_sum:60:python tools/pmc_summary.py $O/o_sq $O/o_fetch $O/o_write --top 40" \
  "r6o/d_sq:200:timeout -s KILL 180 rocprofv3 --pmc $SQ --output-format csv -d $O/d_sq -o run -- $D" \
  "r6o/d_fetch:200:timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/d_fetch -o run -- $D" \
  "r6o/d_write:200:timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/d_write -o run -- $D" \
  "r6o/d_sum:60:python tools/pmc_summary.py $O/d_sq $O/d_fetch $O/d_write --top 40"
