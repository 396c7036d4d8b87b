#!/usr/bin/env python
"""Tiny-BERT AG-News lab entry point (reference `labs/tiny/test_tiny.py`, same CLI) -> mift.apps.tiny_lab.test."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mift.apps.tiny_lab import test  # noqa: E402

if __name__ == "__main__":
    test()
