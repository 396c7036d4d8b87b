#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: every rank binds cuda:0, tensors move over gloo
# (host-staged), exercising the DDP / PP / DP x PP code paths of bench.py end to end.
# The real multi-GPU runs use RCCL ("nccl"); only the transport differs.
export MIFT_BACKEND=gloo
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu_job.sh \
  "rh_ddp2:240:$TR --nproc-per-node 2 --master-port 29611 bench.py --gpus 2 --steps 4 --warmup 2" \
  "rh_pp2:240:PIPELINE_PARALLEL_SIZE=2 $TR --nproc-per-node 2 --master-port 29612 bench.py --gpus 2 --model facebook/opt-125m --pp 2 --micro_batch 8 --steps 3 --warmup 1" \
  "rh_dp2pp2:300:$TR --nproc-per-node 4 --master-port 29613 bench.py --gpus 4 --model facebook/opt-125m --pp 2 --micro_batch 8 --steps 3 --warmup 1" \
  "rh_zero:240:$TR --nproc-per-node 2 --master-port 29614 bench.py --gpus 2 --zero 1 --steps 4 --warmup 2" \
  "torchprof:300:unset MIFT_BACKEND; python bench.py --steps 5 --warmup 3 --profile_dir gpurun_out/torchprof"
