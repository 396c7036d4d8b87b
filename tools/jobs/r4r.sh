#!/bin/bash
# round 4: lora_proj 8-wave blocks (MIFT_LORA_NW A/B) at OPT-2.7B micro-batch 12
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4r
mkdir -p $O
bash tools/gpu_job.sh \
  "r4r/tests:200:MIFT_LORA_NW=8 python -u -m pytest tests/test_kernels_gpu.py -k 'lora_proj' -x -q --timeout 120 --timeout-method thread" \
  "r4r/a_nw4:300:MIFT_LORA_NW=4 python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 3 --warmup 2 --out $O/a_nw4.jsonl" \
  "r4r/a_nw8:300:MIFT_LORA_NW=8 python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 3 --warmup 2 --out $O/a_nw8.jsonl" \
  "r4r/b_nw4:300:MIFT_LORA_NW=4 python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 3 --warmup 2 --out $O/b_nw4.jsonl" \
  "r4r/b_nw8:300:MIFT_LORA_NW=8 python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 3 --warmup 2 --out $O/b_nw8.jsonl" \
  "r4r/kt_nw8:400:MIFT_LORA_NW=8 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 2 --warmup 1 --out $O/kt_nw8.jsonl"
