#!/usr/bin/env python
"""Lab entry point (reference `labs/simple_model/train_simple.py`, same CLI) -> mift.apps.labs.train_simple."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mift.apps.labs import train_simple  # noqa: E402

if __name__ == "__main__":
    train_simple()
