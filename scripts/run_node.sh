#!/bin/bash
# Per-node runner for the OPT LoRA pipeline job (reference: P2/run_node.sh).
#
# Launched once per node by `srun -l scripts/run_node.sh [extra args]` (multi-node) or directly
# (single node).  MI355X-native differences from the reference:
#   * one process per GPU on this node (torchrun --nproc-per-node $NGPU), node rank from
#     SLURM_NODEID and the rendezvous on the first host of the allocation — every rank gets a
#     distinct RANK/WORLD_SIZE (the reference exported neither: all ranks were 0);
#   * the pre-tokenized dataset directory is staged to node-local /tmp once per node
#     (rsync, falling back to cp), as the reference did;
#   * RCCL over xGMI within the node; HSA_ENABLE_IPC_MODE_LEGACY=0 for dmabuf IPC.
set -euo pipefail
cd "$(dirname "$0")/.."

echo "[run_node] host=$(hostname) SLURM_NODEID=${SLURM_NODEID:-0} SLURM_NNODES=${SLURM_NNODES:-1} JOB=${SLURM_JOB_ID:-local}"

MODEL_NAME=${MODEL_NAME:-facebook/opt-2.7b}
DS_CFG=${DS_CFG:-configs/ds_pp_zero1_mi355x.json}
DATA_FILE=${DATA_FILE:-}
SEQ_LEN=${SEQ_LEN:-512} EPOCHS=${EPOCHS:-1} BATCH=${BATCH:-1} ACCUM=${ACCUM:-96} LR=${LR:-5e-5}
LOGDIR=${LOGDIR:-logs/${SLURM_JOB_ID:-local}} OUT_ROOT=${OUT_ROOT:-$HOME/finetuned}
NGPU=${NGPU:-$(python -c 'import torch; print(max(1, torch.cuda.device_count()))' 2>/dev/null || echo 1)}
NNODES=${SLURM_NNODES:-1}
NODE_RANK=${SLURM_NODEID:-0}
if [ -n "${SLURM_JOB_NODELIST:-}" ] && command -v scontrol >/dev/null 2>&1; then
  MASTER_ADDR=${MASTER_ADDR:-$(scontrol show hostnames "$SLURM_JOB_NODELIST" | head -n1)}
fi
MASTER_ADDR=${MASTER_ADDR:-127.0.0.1}
MASTER_PORT=${MASTER_PORT:-29500}

# node-local staging of a pre-tokenized (save_to_disk / npy) dataset directory
if [ -n "$DATA_FILE" ] && [ -d "$DATA_FILE" ]; then
  LOCAL_DS="/tmp/openwebtext_tok_${SLURM_JOB_ID:-local}"
  if [ ! -d "$LOCAL_DS" ]; then
    mkdir -p "$LOCAL_DS"
    if command -v rsync >/dev/null 2>&1; then rsync -a "$DATA_FILE"/ "$LOCAL_DS"/; else cp -r "$DATA_FILE"/. "$LOCAL_DS"/; fi
  fi
  DATA_FILE="$LOCAL_DS"
  echo "[run_node] staged dataset -> $DATA_FILE"
fi

[ -f scripts/env_mi355x.sh ] && source scripts/env_mi355x.sh
export HSA_ENABLE_IPC_MODE_LEGACY=0 TOKENIZERS_PARALLELISM=false
export PIPELINE_PARALLEL_SIZE=${PIPELINE_PARALLEL_SIZE:-$NGPU}
mkdir -p "$LOGDIR"

exec python -m torch.distributed.run --nnodes "$NNODES" --node-rank "$NODE_RANK" --nproc-per-node "$NGPU" \
  --master-addr "$MASTER_ADDR" --master-port "$MASTER_PORT" \
  scripts/finetune_lora_opt_pp.py --model_name "$MODEL_NAME" ${DATA_FILE:+--data_file "$DATA_FILE"} \
  --seq_len "$SEQ_LEN" --epochs "$EPOCHS" --batch "$BATCH" --accum "$ACCUM" --lr "$LR" --ds_cfg "$DS_CFG" \
  --logdir "$LOGDIR" --out_root "$OUT_ROOT" "$@"
