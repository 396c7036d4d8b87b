#!/bin/bash
# Round-3 fourth GPU pass: eager-vs-graph diagnosis (per-parameter), 2dp x 4pp and OPT-6.7B PP8 rehearsals.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
bash tools/gpu_job.sh \
  "d_diag:300:python tools/diag_graph_eager.py --model facebook/opt-125m --precision fp16 --steps 3" \
  "d_dp2pp4:400:python tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 --dp 2 --seq 512 --mb 4 --accum 24 --steps 3" \
  "d_pp8:500:python tools/rehearse_pp.py --model facebook/opt-6.7b --pp 8 --seq 512 --mb 4 --accum 24 --steps 3"
