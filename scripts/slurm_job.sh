#!/bin/bash
# Multi-node template (reference scripts/slurm_job.sh): one torchrun agent per node, 8 GPU ranks each.
#SBATCH -N 2
#SBATCH --ntasks-per-node=1
#SBATCH --gpus-per-node=8
#SBATCH -t 01:00:00
set -euo pipefail
export MASTER_ADDR=$(scontrol show hostnames "$SLURM_JOB_NODELIST" | head -n1) MASTER_PORT=${MASTER_PORT:-29500}
srun bash -c 'NNODES=$SLURM_JOB_NUM_NODES NODE_RANK=$SLURM_NODEID scripts/launch_node.sh "$@"' _ "${@:-bench.py}"
