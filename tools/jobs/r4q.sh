#!/bin/bash
# round 4: lora_proj K-split at OPT's M = 6144 rows (MIFT_LORA_KS A/B), kernel trace of the KS=1 arm
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r4q
mkdir -p $O
bash tools/gpu_job.sh \
  "r4q/a_def:300:python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 3 --warmup 2 --out $O/a_def.jsonl" \
  "r4q/a_ks1:300:MIFT_LORA_KS=1 python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 3 --warmup 2 --out $O/a_ks1.jsonl" \
  "r4q/b_def:300:python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 3 --warmup 2 --out $O/b_def.jsonl" \
  "r4q/b_ks1:300:MIFT_LORA_KS=1 python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 3 --warmup 2 --out $O/b_ks1.jsonl" \
  "r4q/kt_ks1:400:MIFT_LORA_KS=1 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/mb_sweep.py --model facebook/opt-2.7b --mbs 12 --steps 2 --warmup 1 --out $O/kt_ks1.jsonl"
