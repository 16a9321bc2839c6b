import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, 'tests', 'golden')
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (HIP device); run with -m gpu')
    config.addinivalue_line('markers', 'slow: long-running test')


def pytest_collection_finish(session):
    """A GPU session initialises torch's HIP runtime before any library context: torch bundles its own
    runtime, which finds no device when this library's runtime came up first in the process (the
    reverse order works).  Tests that mix both then run in any order or subset."""
    if not any(item.get_closest_marker('gpu') for item in session.items):
        return
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.device_count() > 0:
        torch.cuda.init()
