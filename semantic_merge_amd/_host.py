"""Loader of the native host module ``_smx_host.so`` (csrc/smx_host.cpp, built by
csrc/Makefile).  The drop-in's marshal / materialise run there; a missing build fails
loudly instead of falling back to the Python restatement."""
from __future__ import annotations

import importlib
import os

_mod = None


def host():
    global _mod
    if _mod is None:
        here = os.path.dirname(os.path.abspath(__file__))
        if not os.path.exists(os.path.join(here, "_smx_host.so")):
            raise ImportError("semantic_merge_amd/_smx_host.so is not built: run "
                              "`make -C semantic_merge_amd/csrc` (or __graft_entry__.build())")
        _mod = importlib.import_module(".._smx_host", __name__)
    return _mod
