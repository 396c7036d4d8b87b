#!/usr/bin/env bash
# Multi-node lab launcher (reference labs/tiny/side_shell_pr.sh, which GENERATES ~/launch_tiny.sh).
#
#   ACTION=train bash scripts/launch_tiny.sh [--subset 2000 --epochs 1 --batch 8]
#   ACTION=infer bash scripts/launch_tiny.sh --ckpt ./tiny_out
#   bash scripts/launch_tiny.sh --write ~/launch_tiny.sh     # reference-style: emit a standalone copy
#
# Flow (same contract as the reference launcher):
#   1. outside a SLURM allocation -> re-run itself under `salloc $SALLOC_OPTS`;
#   2. rendezvous endpoint = first host of the nodelist (c10d, --rdzv-id=$SLURM_JOB_ID);
#   3. preflight: every node must see the project dir; if not, tar it and `sbcast` it to /tmp/<job>/ and run there;
#   4. per-node sanity banner (NODE <host> OK -> PY ... torch ... tfm ... numpy ...);
#   5. `srun` one torchrun per node: --nnodes=$SLURM_NNODES --nproc-per-node=$GPUS_PER_NODE --node-rank=$SLURM_NODEID,
#      which dispatches ACTION (train|infer|test|eval|simple|finetune|transfer|rag|gen) through mift.apps.run_action.
# MI355X-first: one rank per GPU (GPUS_PER_NODE defaults to the node's visible GPUs, 8 on an MI355X node), RCCL over
# xGMI inside a node; the reference ran 2 CPU ranks per node over gloo.
# Env: ACTION, EXTRA_ARGS, SALLOC_OPTS, GPUS_PER_NODE, MASTER_PORT, DEBUG=1 (set -x)
set -Eeuo pipefail
trap 'echo "[launch_tiny] FAILED at line $LINENO rc=$?" >&2' ERR
[[ "${DEBUG:-0}" == 1 ]] && set -x

SELF="$(readlink -f "${BASH_SOURCE[0]}")"
ROOT="$(cd "$(dirname "$SELF")/.." && pwd)"

if [[ "${1:-}" == "--write" ]]; then
  dst="${2:?--write <path>}"
  sed "s#^ROOT=.*#ROOT=\"$ROOT\"#" "$SELF" > "$dst" && chmod +x "$dst"
  echo "wrote $dst (project root $ROOT)"; exit 0
fi

ACTION="${ACTION:-train}"
if [[ -z "${SLURM_JOB_ID:-}" ]]; then
  if command -v salloc >/dev/null 2>&1; then
    # shellcheck disable=SC2086
    exec salloc ${SALLOC_OPTS:---nodes=2 --ntasks-per-node=1 --gpus-per-node=8 --time=00:30:00} \
      env ACTION="$ACTION" EXTRA_ARGS="${EXTRA_ARGS:-}" bash "$SELF" "$@"
  fi
  echo "[launch_tiny] no SLURM: single-node run" >&2
  SLURM_JOB_ID="local$(date +%s)"; SLURM_NNODES=1; SLURM_JOB_NODELIST="$(hostname)"; LOCAL_ONLY=1
fi

hosts() { if [[ "${LOCAL_ONLY:-0}" == 1 ]]; then hostname; else scontrol show hostnames "$SLURM_JOB_NODELIST"; fi; }
MASTER_ADDR="$(hosts | head -n1)"
[[ "${LOCAL_ONLY:-0}" == 1 ]] && MASTER_ADDR=127.0.0.1
MASTER_PORT="${MASTER_PORT:-$((29500 + ${SLURM_JOB_ID//[!0-9]/} % 1000))}"
NNODES="${SLURM_NNODES:-1}"
GPUS_PER_NODE="${GPUS_PER_NODE:-$(python -c 'import torch; print(max(1, torch.cuda.device_count()))')}"

# preflight: does every node see the project directory?
RUN_ROOT="$ROOT"
if [[ "${LOCAL_ONLY:-0}" != 1 ]]; then
  if ! srun --ntasks-per-node=1 test -r "$ROOT/mift/__init__.py"; then
    echo "[launch_tiny] project not visible on all nodes -> staging with sbcast"
    tarball="/tmp/mift_${SLURM_JOB_ID}.tar"
    tar -C "$(dirname "$ROOT")" -cf "$tarball" --exclude=.git --exclude=gpurun_out "$(basename "$ROOT")"
    sbcast -f "$tarball" "$tarball"
    srun --ntasks-per-node=1 bash -c "mkdir -p /tmp/mift_$SLURM_JOB_ID && tar -C /tmp/mift_$SLURM_JOB_ID -xf $tarball"
    RUN_ROOT="/tmp/mift_${SLURM_JOB_ID}/$(basename "$ROOT")"
  fi
fi

# per-node environment (offline HF, RCCL/gloo, threads)
export ACTION MASTER_ADDR MASTER_PORT HSA_ENABLE_IPC_MODE_LEGACY=0 TOKENIZERS_PARALLELISM=false
export HF_HUB_OFFLINE=1 HF_DATASETS_OFFLINE=1 TRANSFORMERS_OFFLINE=1 OMP_NUM_THREADS="${OMP_NUM_THREADS:-8}"
export PYTHONPATH="$RUN_ROOT${PYTHONPATH:+:$PYTHONPATH}"

node_cmd() {  # $1 = node rank
  echo "torchrun: nnodes=$NNODES nproc_per_node=$GPUS_PER_NODE node_rank=$1 rdzv=$MASTER_ADDR:$MASTER_PORT"
  cd "$RUN_ROOT"
  python -m mift.apps.run_action --sanity
  # shellcheck disable=SC2086
  python -m torch.distributed.run --nnodes "$NNODES" --nproc-per-node "$GPUS_PER_NODE" \
    --rdzv-backend c10d --rdzv-endpoint "$MASTER_ADDR:$MASTER_PORT" --rdzv-id "$SLURM_JOB_ID" \
    --node-rank "$1" -m mift.apps.run_action ${EXTRA_ARGS:-} "${@:2}"
}

if [[ "${LOCAL_ONLY:-0}" == 1 ]]; then
  node_cmd 0 "$@"
else
  export -f node_cmd
  export NNODES GPUS_PER_NODE RUN_ROOT EXTRA_ARGS SLURM_JOB_ID
  srun --ntasks-per-node=1 --kill-on-bad-exit=1 bash -c 'node_cmd "$SLURM_NODEID" "$@"' _ "$@"
fi
echo "Usage: ACTION=train|infer|test|eval bash scripts/launch_tiny.sh [args]  (EXTRA_ARGS, SALLOC_OPTS, GPUS_PER_NODE)"
