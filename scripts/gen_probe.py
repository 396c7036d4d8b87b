#!/usr/bin/env python
"""Greedy generation probe (reference run_labs45_tiny_final.sbatch:66-89) -> mift.apps.gen_probe."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mift.apps.gen_probe import main  # noqa: E402

if __name__ == "__main__":
    main()
