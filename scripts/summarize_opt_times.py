#!/usr/bin/env python
"""Max [Training] seconds over ranks per log dir (reference summarize_opt_times.py CLI)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mift.obs.logparse import summarize_times  # noqa: E402

if __name__ == "__main__":
    if len(sys.argv) < 2:
        print("Usage: python summarize_opt_times.py logs/<JOBID> [logs/<JOBID> ...]")
        sys.exit(1)
    print(summarize_times(sys.argv[1:], "OPT-2.7B LoRA — PP + ZeRO-1 Training Times"))
