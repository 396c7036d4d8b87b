"""Per-node action wrapper for the multi-node lab launcher.

Reference: ``labs/tiny/side_shell_pr.sh:92-182`` writes a ``_sanity.py`` (per-node
version banner) and a ``_run_wrapper.py`` that patches ``datasets`` for NumPy 2
and dispatches ``ACTION=train|infer`` to the lab scripts with ``runpy``.

Here one module does both: ``python -m mift.apps.run_action [--sanity] [args...]``
prints the ``NODE <host> OK -> PY … torch … tfm … numpy … datasets …`` line
(parsed by ``labs/tiny/eval_logs.py``) and runs the action's script in-process
with ``sys.argv`` rewritten, so torchrun's per-rank env reaches it unchanged.
No NumPy-2 patch is needed: the pinned ``datasets`` already supports NumPy 2.
"""
import os
import runpy
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ACTIONS = {
    "train": "labs/tiny/train_tiny.py",
    "infer": "labs/tiny/infer_ddp.py",
    "test": "labs/tiny/test_tiny.py",
    "eval": "labs/tiny/eval_logs.py",
    "simple": "labs/simple_model/train_simple.py",
    "finetune": "labs/fine_tuning/fine_tune.py",
    "transfer": "labs/transfer_learning/transfer.py",
    "rag": "labs/ragging/rag_example.py",
    "gen": "scripts/gen_probe.py",
}


def sanity_line() -> str:
    import numpy
    import torch
    try:
        import transformers
        tv = transformers.__version__
    except Exception:  # noqa: BLE001
        tv = "NA"
    try:
        import datasets
        dv = datasets.__version__
    except Exception:  # noqa: BLE001
        dv = "NA"
    return (f"NODE {socket.gethostname()} OK -> PY {sys.version.split()[0]} torch {torch.__version__} tfm {tv} "
            f"numpy {numpy.__version__} datasets {dv} root {os.getcwd()}")


def resolve(action: str) -> str:
    if action not in ACTIONS:
        raise SystemExit(f"Unknown ACTION={action!r}; expected one of {sorted(ACTIONS)}")
    return os.path.join(ROOT, ACTIONS[action])


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv[:1] == ["--sanity"]:
        print(sanity_line(), flush=True)
        return 0
    action = os.environ.get("ACTION", "train")
    script = resolve(action)
    if os.environ.get("LOCAL_RANK", "0") == "0":
        print(sanity_line(), flush=True)
    sys.argv = [script] + argv
    sys.path.insert(0, os.path.dirname(script))
    runpy.run_path(script, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main())
