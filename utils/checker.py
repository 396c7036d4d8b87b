#!/usr/bin/env python
"""Cluster tool (reference `utils/checker.py`) -> mift.utils.cluster.main_checker."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mift.utils.cluster import main_checker  # noqa: E402

if __name__ == "__main__":
    sys.exit(main_checker() and 0)
