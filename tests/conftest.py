"""pytest configuration: registers the `gpu` marker.

CPU tier:  python -m pytest tests/ -x -q -m "not gpu"
GPU tier:  python -m pytest tests/ -x -q -m gpu   (needs a real MI355X)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import pytest  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True, scope="session")
def _destroy_process_groups():
    """Tests that form a single-process world (gloo / RCCL, world 1) leave the default group alive for
    the next test; tear it down once at the end so the run exits without the 'destroy_process_group()
    was not called' resource-leak warning."""
    yield
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # pragma: no cover - best effort at interpreter shutdown
        pass
