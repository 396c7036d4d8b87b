#!/usr/bin/env python
"""Cluster tool (reference `utils/Connect2Cluster.py`) -> mift.utils.cluster.connect."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mift.utils.cluster import connect  # noqa: E402

if __name__ == "__main__":
    sys.exit(connect() and 0)
