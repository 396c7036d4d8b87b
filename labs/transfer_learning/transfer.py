#!/usr/bin/env python
"""Lab entry point (reference `labs/transfer_learning/transfer.py`, same CLI) -> mift.apps.labs.transfer."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mift.apps.labs import transfer  # noqa: E402

if __name__ == "__main__":
    transfer()
