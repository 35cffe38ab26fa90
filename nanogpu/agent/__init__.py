"""MI355X node agent: topology publisher + kubelet device plugin (see node.py, plugin.py)."""
from __future__ import annotations

__all__ = ["main"]


def main(argv=None) -> int:
    from .node import main as _main

    return _main(argv)
