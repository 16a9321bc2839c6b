"""A module imported on first attribute access.

pandas costs ~0.5 s to import; the columnar CLI path (fastcli.py) reads, clusters and writes without
it, so the modules that use pandas on the other paths (the DataFrame entry points of cluster.py, the
pandas I/O of main.py and ingest.py) reach it through this proxy.
"""
from __future__ import annotations

import importlib


class LazyModule:
    def __init__(self, name: str):
        self._name = name
        self._mod = None

    def __getattr__(self, attr):
        if self._mod is None:
            self._mod = importlib.import_module(self._name)
        return getattr(self._mod, attr)


pandas = LazyModule('pandas')
