#!/usr/bin/env python
"""Tiny-BERT AG-News lab entry point (reference `labs/tiny/infer_ddp.py`, same CLI) -> mift.apps.tiny_lab.infer."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mift.apps.tiny_lab import infer  # noqa: E402

if __name__ == "__main__":
    infer()
