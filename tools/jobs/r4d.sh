#!/bin/bash
# round 4 (after the first sweep): fixed bench + single-command PP rehearsal, full GPU suite, generation
# probes (eager vs graphed decode), GEMM tile experiments, eager-vs-graph diagnostic for distilgpt2
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r4d
bash tools/gpu_job.sh \
  "r4d/bench:300:python bench.py --steps 20 --warmup 5" \
  "r4d/bench_cfg3_gloo:500:MIFT_BACKEND=gloo python bench.py --gpus 4 --config 3 --steps 2 --warmup 1" \
  "r4d/pytest:900:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r4d/gen_eager:200:MIFT_GEN_GRAPH=0 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4d/gen_graph:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4d/gen_graph_distinct:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5 --prompts distinct" \
  "r4d/dgpt_tiles:400:MIFT_EXT_SO=.wip/_C_exp.so TILES=0,7,9,10,11,12 python tools/bench_kernels.py --only dgpt --json gpurun_out/r4d/dgpt_tiles.json" \
  "r4d/optm_tiles:600:MIFT_EXT_SO=.wip/_C_exp.so TILES=0,3,6,8,10,11,12 python tools/bench_kernels.py --only optm --json gpurun_out/r4d/optm_tiles.json" \
  "r4d/diag_graph:400:python tools/diag_graph_eager.py --model distilgpt2 --precision bf16 --steps 20" \
  "r4d/rehearse_pp4v4:700:python tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 --virtual 4 --mb 12 --accum 8 --steps 3 > gpurun_out/r4d/rehearse_opt27b_pp4v4.json"
