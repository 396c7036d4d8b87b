#!/usr/bin/env python
"""Evaluate a multi-rank run from its logs (reference `labs/tiny/eval_logs.py` CLI:
``--job ID [--logs-dir ~/slurm_logs]``, globs ``*.{ID}.*.out``) -> mift.obs.logparse."""
import argparse
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mift.obs.logparse import evaluate_logs, format_report  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--job", required=True)
    ap.add_argument("--logs-dir", default=os.path.expanduser("~/slurm_logs"))
    a = ap.parse_args()
    outs = sorted(glob.glob(os.path.join(a.logs_dir, f"*.{a.job}.*.out")))
    if not outs:
        print(f"[!] No log files found matching {a.logs_dir}/*.{a.job}.*.out", file=sys.stderr)
        sys.exit(2)
    r = evaluate_logs(outs, preflight=os.path.join(a.logs_dir, f"preflight.{a.job}.txt"))
    print(format_report(r, a.job))


if __name__ == "__main__":
    main()
