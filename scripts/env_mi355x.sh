#!/usr/bin/env bash
# Source me:  source scripts/env_mi355x.sh
# Environment activator + import probe for MI355X nodes (reference P1/venv_env.sh:1-58).
#
# Reference: activates /opt/llamaenv or ~/llamaenv_local (exit 90 when neither exists), sets a CPU-only Gloo env and
# HF caches, then probes torch/transformers/datasets/peft imports.
# Here: the Python env is optional (ROCm images ship torch system-wide); the comm env is RCCL over xGMI (gloo only as
# the control plane); the probe checks that the gfx950 extension (_C.so) loads and sees the GPUs.
#   MIFT_VENV      venv to activate (else $HOME/mift_venv if present, else the system python)
#   MIFT_REQUIRE_VENV=1  exit 90 when no venv was found (reference behaviour)
#   MIFT_PROBE=0   skip the import probe
_mift_root="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
_mift_fail() { echo "[env] $*" >&2; return 90 2>/dev/null || exit 90; }

for _v in "${MIFT_VENV:-}" "$HOME/mift_venv"; do
  if [[ -n "$_v" && -f "$_v/bin/activate" ]]; then
    # shellcheck disable=SC1091
    source "$_v/bin/activate"; echo "[env] venv: $_v"; break
  fi
done
if [[ "${MIFT_REQUIRE_VENV:-0}" == 1 && -z "${VIRTUAL_ENV:-}" ]]; then _mift_fail "no venv found (MIFT_VENV, ~/mift_venv)"; fi

# communication: RCCL over xGMI for tensors, gloo for control traffic
export HSA_ENABLE_IPC_MODE_LEGACY=0            # dmabuf IPC (required by the host driver)
export TORCH_NCCL_ASYNC_ERROR_HANDLING="${TORCH_NCCL_ASYNC_ERROR_HANDLING:-1}"
export NCCL_IB_DISABLE="${NCCL_IB_DISABLE:-1}"  # single node: xGMI only
export GLOO_SOCKET_TIMEOUT="${GLOO_SOCKET_TIMEOUT:-600}"
export MIFT_COMM_TIMEOUT="${MIFT_COMM_TIMEOUT:-1800}"
export OMP_NUM_THREADS="${OMP_NUM_THREADS:-8}" TOKENIZERS_PARALLELISM=false
# offline HF caches (no network on compute nodes)
export HF_HOME="${HF_HOME:-$_mift_root/.hf_cache}"
export HF_DATASETS_CACHE="${HF_DATASETS_CACHE:-$HF_HOME/ds}" TRANSFORMERS_CACHE="${TRANSFORMERS_CACHE:-$HF_HOME/hub}"
export HF_HUB_OFFLINE=1 HF_DATASETS_OFFLINE=1 TRANSFORMERS_OFFLINE=1
export PYTHONPATH="$_mift_root${PYTHONPATH:+:$PYTHONPATH}"

if [[ "${MIFT_PROBE:-1}" == 1 ]]; then
  python - <<'PY' || _mift_fail "import probe failed"
import importlib, sys
ok = True
for m in ("numpy", "torch", "transformers", "datasets", "safetensors"):
    try:
        mod = importlib.import_module(m)
        print(f"[env] {m:12s} {getattr(mod, '__version__', '?')}")
    except Exception as e:  # noqa: BLE001
        print(f"[env] {m:12s} MISSING ({e})"); ok = ok and m not in ("numpy", "torch")
import torch
n = torch.cuda.device_count()
print(f"[env] gpus visible: {n}")
try:
    from mift import _ext
    _ext.require()
    print("[env] mift._C    loaded (gfx950)")
except Exception as e:  # noqa: BLE001
    print(f"[env] mift._C    NOT loaded ({e}); run: python -m mift.build")
    ok = ok and n == 0
sys.exit(0 if ok else 1)
PY
fi
unset _v _mift_root
