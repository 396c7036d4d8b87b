#!/bin/bash
# round 4: K-split skinny decode GEMM (fc2), decode_tail bookkeeping prefetch; decode + per-op traces
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4n
mkdir -p $O
bash tools/gpu_job.sh \
  "r4n/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_infer_gpu.py -k 'skinny or decode or infer or generate or padded or graphed or gemm_ln or splitk' -x -q --timeout 120 --timeout-method thread" \
  "r4n/gen_graph:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4n/gen_graph_distinct:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5 --prompts distinct" \
  "r4n/gen_eager:200:MIFT_GEN_GRAPH=0 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4n/kt_decode:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktdec -o run -- python3 scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 3"
