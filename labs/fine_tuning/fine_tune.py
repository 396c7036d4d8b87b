#!/usr/bin/env python
"""Lab entry point (reference `labs/fine_tuning/fine_tune.py`, same CLI) -> mift.apps.labs.fine_tune."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mift.apps.labs import fine_tune  # noqa: E402

if __name__ == "__main__":
    fine_tune()
