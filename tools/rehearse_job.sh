#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: every rank binds cuda:0, tensors move over gloo
# (host-staged), exercising the DDP / PP / DP x PP / ZeRO-1 code paths of bench.py end to end
# (including the wall-clock/epoch pass on a small corpus).  The real multi-GPU runs use RCCL
# ("nccl"); only the transport differs.
export MIFT_BACKEND=gloo
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu_job.sh \
  "rh_ddp2:240:$TR --nproc-per-node 2 --master-port 29611 bench.py --gpus 2 --steps 4 --warmup 2 --epoch_lines 640" \
  "rh_pp2:240:PIPELINE_PARALLEL_SIZE=2 $TR --nproc-per-node 2 --master-port 29612 bench.py --gpus 2 --model facebook/opt-125m --pp 2 --micro_batch 8 --steps 3 --warmup 1" \
  "rh_dp2pp2:300:$TR --nproc-per-node 4 --master-port 29613 bench.py --gpus 4 --model facebook/opt-125m --pp 2 --micro_batch 8 --steps 3 --warmup 1" \
  "rh_zero:240:$TR --nproc-per-node 2 --master-port 29614 bench.py --gpus 2 --zero 1 --steps 4 --warmup 2 --epoch_lines 0" \
  "rh_p1prof:300:$TR --nproc-per-node 2 --master-port 29615 scripts/finetune_lora_distilgpt2.py --dataset medium --synthetic 2048 --max_steps 8 --logging_steps 4 --no_save --logdir gpurun_out/p1prof/logs --out_root gpurun_out/p1prof/out --profile gpurun_out/p1prof/trace --profile_steps 4:7"
