#!/usr/bin/env bash
# Offline wheel staging (reference labs/tiny/req.sh:1-40).
#   bash scripts/stage_wheels.sh download [DIR]   # on a node WITH network: fetch wheels of requirements.txt into DIR
#   bash scripts/stage_wheels.sh install  [DIR]   # on compute nodes WITHOUT network: install from DIR only
# DIR defaults to $OFFLINE_ROOT/pkgs (OFFLINE_ROOT defaults to the project root).  torch is taken from the ROCm
# index; nothing is ever built from source on a compute node.
set -Eeuo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
MODE="${1:?usage: stage_wheels.sh download|install [DIR]}"
DIR="${2:-${OFFLINE_ROOT:-$ROOT}/pkgs}"
mkdir -p "$DIR"
case "$MODE" in
  download)
    python -m pip download -d "$DIR" --only-binary=:all: \
      --extra-index-url "${TORCH_INDEX:-https://download.pytorch.org/whl/rocm7.0}" -r "$ROOT/requirements.txt" ;;
  install)
    python -m pip install --no-index --find-links "$DIR" -r "$ROOT/requirements.txt" ;;
  *) echo "unknown mode $MODE" >&2; exit 2 ;;
esac
echo "[stage_wheels] $MODE done ($DIR)"
