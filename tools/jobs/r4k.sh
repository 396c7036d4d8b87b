#!/bin/bash
# round 4: decode (skinny GEMM N<=4096/K<=1024, LN prologue, batched decode_tail), full GPU suite,
# bench; experimental whole-sequence attention forward with next-tile K prefetch (A/B, .wip build)
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4k
mkdir -p $O
X="MIFT_EXT_SO=.wip/_C_exp.so"
bash tools/gpu_job.sh \
  "r4k/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_infer_gpu.py -k 'skinny or decode or infer or generate or padded or graphed or gemm_ln or lora_proj' -x -q --timeout 120 --timeout-method thread" \
  "r4k/gen_graph:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4k/tests_skinny2:300:MIFT_GEMM_SKINNY=2 python -u -m pytest tests/test_kernels_gpu.py tests/test_infer_gpu.py -k 'skinny or graphed or padded' -x -q --timeout 120 --timeout-method thread" \
  "r4k/gen_graph_skinny2:200:MIFT_GEMM_SKINNY=2 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4k/kt_decode_skinny2:200:MIFT_GEMM_SKINNY=2 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktdec2 -o run -- python3 scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 3" \
  "r4k/gen_graph_distinct:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5 --prompts distinct" \
  "r4k/gen_eager:200:MIFT_GEN_GRAPH=0 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4k/kt_decode:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktdec -o run -- python3 scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 3" \
  "r4k/tests_pf:300:$X MIFT_ATTN_PF=1 python -u -m pytest tests/test_kernels_gpu.py -k 'attention or attn' -x -q --timeout 120 --timeout-method thread" \
  "r4k/a_pf0:200:$X MIFT_ATTN_PF=0 python tools/bench_attn.py" \
  "r4k/a_pf1:200:$X MIFT_ATTN_PF=1 python tools/bench_attn.py" \
  "r4k/b_pf0:200:$X MIFT_ATTN_PF=0 python tools/bench_attn.py" \
  "r4k/b_pf1:200:$X MIFT_ATTN_PF=1 python tools/bench_attn.py" \
  "r4k/dgpt_tiles:400:$X TILES=0,13,7,15,9,14 python tools/bench_kernels.py --only dgpt --json $O/dgpt_tiles.json" \
  "r4k/mb_sweep:600:python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 4,8,12,16,24,48 --out $O/mb_sweep_opt27b.jsonl" \
  "r4k/pytest:900:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r4k/bench:300:python bench.py --steps 20 --warmup 5"
