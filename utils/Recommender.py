#!/usr/bin/env python
"""Cluster tool (reference `utils/Recommender.py`) -> mift.utils.cluster.main_recommender."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mift.utils.cluster import main_recommender  # noqa: E402

if __name__ == "__main__":
    sys.exit(main_recommender() and 0)
