#!/usr/bin/env bash
# One MI355X node, one process per GPU (torchrun), RCCL over xGMI.
# Shared launcher behind the sbatch wrappers (reference contract: P1/submit_distilgpt2_lora.sbatch,
# SURVEY C01/C02/A.2): env knobs, ERR trap, structured exit codes, preflight, sanity banner,
# meta.json / meta.final.json / wallclock_seconds.txt in $LOGDIR.
#
#   scripts/launch_node.sh <entry.py> [args...]      e.g. scripts/launch_node.sh scripts/finetune_lora_distilgpt2.py --dataset medium
# Env: NGPU (default: all visible), MASTER_ADDR/MASTER_PORT, LOGDIR, OUT_ROOT, DATA_FILE, DATASET, SEQ_LEN, EPOCHS,
#      BATCH, ACCUM, LR, OMP_NUM_THREADS, PIPELINE_PARALLEL_SIZE, NNODES/NODE_RANK (multi-node torchrun)
set -Eeuo pipefail
trap 'echo "[FATAL] line $LINENO rc=$?" >&2' ERR
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
ENTRY="${1:?usage: launch_node.sh <entry.py> [args...]}"; shift
[[ -f "$ENTRY" ]] || { echo "ERROR: entry script missing: $ENTRY" >&2; exit 11; }

NGPU="${NGPU:-$(python - <<'PY'
import torch; print(max(1, torch.cuda.device_count()))
PY
)}"
export MASTER_ADDR="${MASTER_ADDR:-127.0.0.1}" MASTER_PORT="${MASTER_PORT:-29500}"
export NNODES="${NNODES:-${SLURM_NNODES:-1}}" NODE_RANK="${NODE_RANK:-${SLURM_NODEID:-0}}"
export JOB_ID="${JOB_ID:-${SLURM_JOB_ID:-local$(date +%s)}}"
export LOGDIR="${LOGDIR:-$ROOT/logs/$JOB_ID}" OUT_ROOT="${OUT_ROOT:-$HOME/finetuned}"
export OMP_NUM_THREADS="${OMP_NUM_THREADS:-8}" TOKENIZERS_PARALLELISM=false
export HSA_ENABLE_IPC_MODE_LEGACY=0
export GLOO_SOCKET_TIMEOUT="${GLOO_SOCKET_TIMEOUT:-1800}"
mkdir -p "$LOGDIR" "$OUT_ROOT"

# preflight (reference exit codes 21/22/23)
if [[ -n "${DATA_FILE:-}" && ! -r "$DATA_FILE" && "${ALLOW_SYNTHETIC:-1}" != 1 ]]; then
  echo "[Preflight] Cannot read dataset: $DATA_FILE" >&2; exit 22; fi
[[ -w "$OUT_ROOT" ]] || { echo "[Preflight] OUT_ROOT not writable: $OUT_ROOT" >&2; exit 23; }

# sanity banner (parsed by eval_logs.py) + import probe (exit 34)
python - <<'PY' || { echo "[Launch] python import failed" >&2; exit 34; }
import os, socket, sys, numpy, torch
try:
    import transformers as t; tv = t.__version__
except Exception:
    tv = "NA"
try:
    import datasets as d; dv = d.__version__
except Exception:
    dv = "NA"
print(f"NODE {socket.gethostname()} OK -> PY {sys.version.split()[0]} torch {torch.__version__} tfm {tv} "
      f"numpy {numpy.__version__} datasets {dv} root {os.getcwd()}", flush=True)
PY

python - "$LOGDIR/meta.json" "$NNODES" "$NGPU" <<'PY'
import json, os, sys
keys = ["DATASET", "DATA_FILE", "SEQ_LEN", "EPOCHS", "BATCH", "ACCUM", "LR", "PIPELINE_PARALLEL_SIZE",
        "MASTER_ADDR", "MASTER_PORT", "JOB_ID"]
meta = {k.lower(): os.environ[k] for k in keys if k in os.environ}
meta.update({"nnodes": int(sys.argv[2]), "gpus_per_node": int(sys.argv[3]),
             "world_size": int(sys.argv[2]) * int(sys.argv[3]), "job_id": os.environ["JOB_ID"]})
json.dump(meta, open(sys.argv[1], "w"), indent=2)
PY

echo "torchrun: nnodes=$NNODES nproc_per_node=$NGPU node_rank=$NODE_RANK rdzv=$MASTER_ADDR:$MASTER_PORT"
T0=$(date +%s)
set +e
python -m torch.distributed.run --nnodes "$NNODES" --node-rank "$NODE_RANK" --nproc-per-node "$NGPU" \
  --master-addr "$MASTER_ADDR" --master-port "$MASTER_PORT" "$ENTRY" "$@"
RC=$?
set -e
WALL=$(( $(date +%s) - T0 ))
echo "$WALL" > "$LOGDIR/wallclock_seconds.txt"
python - "$LOGDIR" "$RC" "$WALL" <<'PY'
import json, os, sys
d, rc, wall = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
m = json.load(open(os.path.join(d, "meta.json")))
m.update({"status": "success" if rc == 0 else "failure", "wall_seconds": wall, "rc": rc})
json.dump(m, open(os.path.join(d, "meta.final.json"), "w"), indent=2)
PY
echo "[JOB] completed: logs=$LOGDIR wall=${WALL}s status=$([ "$RC" -eq 0 ] && echo OK || echo FAIL) (rc=$RC)"
exit "$RC"
