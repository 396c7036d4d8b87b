#!/bin/bash
# Round-3 fifth GPU pass: MFMA row-projection kernels (tests + bench + step), then the pack-generation
# fix — eager-vs-graph diag, graph/pipeline tests, the three BASELINE PP rehearsals.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
bash tools/gpu_job.sh \
  "e_rp_tests:200:python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k 'rowproj or lora_proj'" \
  "e_rp_bench:200:python tools/bench_rowproj.py" \
  "e_bench:300:python bench.py --epoch_lines 0" \
  "e_kt:240:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0" \
  "e_diag:300:python tools/diag_graph_eager.py --model facebook/opt-125m --precision fp16 --steps 3" \
  "e_tests:400:python -u -m pytest tests/test_graph_gpu.py tests/test_pipeline_gpu.py -q --timeout 300 --timeout-method thread" \
  "e_pp4:300:python tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 --seq 512 --mb 4 --accum 24 --steps 3" \
  "e_dp2pp4:300:python tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 --dp 2 --seq 512 --mb 4 --accum 24 --steps 3" \
  "e_pp8:400:python tools/rehearse_pp.py --model facebook/opt-6.7b --pp 8 --seq 512 --mb 4 --accum 24 --steps 3"
