#!/bin/bash
# round 4: skinny decode GEMM limited to N<=4096,K<=1024; batched decode_tail; full GPU suite
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4i
mkdir -p $O
bash tools/gpu_job.sh \
  "r4i/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_infer_gpu.py -k 'skinny or decode or infer or generate or padded or graphed or gemm_ln' -x -q --timeout 120 --timeout-method thread" \
  "r4i/gen_graph:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4i/gen_graph_distinct:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5 --prompts distinct" \
  "r4i/gen_eager:200:MIFT_GEN_GRAPH=0 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4i/kt_decode:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktdec -o run -- python3 scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 3" \
  "r4i/pytest:900:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r4i/bench:300:python bench.py --steps 20 --warmup 5"
