#!/usr/bin/env python
"""RAG demo entry point (reference `labs/ragging/rag_example.py`, same CLI) -> mift.apps.rag."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mift.apps.rag import main  # noqa: E402

if __name__ == "__main__":
    main()
