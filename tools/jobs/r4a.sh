#!/bin/bash
# round 4, first GPU call: GPU suite, flagship bench, single-command PP rehearsal, micro-batch sweeps,
# OPT-2.7B kernel traces at the PP micro-batch (4) and the dp1 one (48).
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r4a
bash tools/gpu_job.sh \
  "r4a/pytest:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r4a/bench:300:python bench.py --steps 20 --warmup 5" \
  "r4a/bench_cfg3_gloo:400:MIFT_BACKEND=gloo python bench.py --gpus 4 --config 3 --steps 2 --warmup 1" \
  "r4a/mb_sweep_27:500:python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 1,2,4,8,12,16,24,48 --steps 2 --warmup 1 --out gpurun_out/r4a/mb_sweep_opt27b.jsonl" \
  "r4a/mb_sweep_67:500:python tools/mb_sweep.py --model facebook/opt-6.7b --mbs 1,2,4,8,16,32 --steps 2 --warmup 1 --out gpurun_out/r4a/mb_sweep_opt67b.jsonl" \
  "r4a/kt_opt_mb4:300:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4a/kt_mb4 -o run -- python3 bench.py --model facebook/opt-2.7b --micro_batch 4 --steps 2 --warmup 1" \
  "r4a/kt_opt_mb48:300:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4a/kt_mb48 -o run -- python3 bench.py --model facebook/opt-2.7b --micro_batch 48 --steps 2 --warmup 1"
