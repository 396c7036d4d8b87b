#!/bin/bash
# Round-3 sweep of every entry point on one MI355X (multi-rank ones over gloo, every rank on cuda:0):
# P2 app (PP2 + ZeRO-1 from the DS config, recompute arm, save), P1 app resume, the labs, RAG.
export MIFT_BACKEND=gloo
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=/tmp/apps  # checkpoints stay on the box (the merge back is capped at 64 MiB); logs: gpurun_out/<step>.log
mkdir -p $O
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu_job.sh \
  "a_p2pp2:300:PIPELINE_PARALLEL_SIZE=2 $TR --nproc-per-node 2 --master-port 29621 scripts/finetune_lora_opt_pp.py --model_name facebook/opt-125m --data_file none.txt --synthetic 512 --seq_len 256 --accum 8 --max_steps 4 --log_every 1 --logdir $O/p2_logs --out_root $O/p2_out" \
  "a_p2ckpt:300:PIPELINE_PARALLEL_SIZE=2 $TR --nproc-per-node 2 --master-port 29622 scripts/finetune_lora_opt_pp.py --model_name facebook/opt-125m --data_file none.txt --synthetic 512 --seq_len 256 --accum 8 --max_steps 3 --log_every 1 --gradient_checkpointing 1 --logdir $O/p2c_logs --out_root $O/p2c_out" \
  "a_p1ckpt:300:python scripts/finetune_lora_distilgpt2.py --dataset medium --synthetic 2048 --max_steps 12 --save_steps 6 --logging_steps 6 --logdir $O/p1_logs --out_root $O/p1_out" \
  "a_tiny:300:python labs/tiny/train_tiny.py --subset 512 --epochs 1 --batch 8 --out $O/tiny_out --no_tb && python labs/tiny/test_tiny.py --ckpt $O/tiny_out && python labs/tiny/infer_ddp.py --ckpt $O/tiny_out --max_test 256" \
  "a_simple:200:python labs/simple_model/train_simple.py --max_steps 4 --output_dir $O/simple" \
  "a_ft:200:python labs/fine_tuning/fine_tune.py --max_steps 8 --output_dir $O/ft" \
  "a_tl:400:python labs/transfer_learning/transfer.py --epochs 1 --output_dir $O/tl" \
  "a_rag:200:python labs/ragging/rag_example.py --subset 200 --max_new_tokens 8"
