"""Native data plane loader.

``load()`` returns the compiled ``_kgs_native`` module, building it in-tree first
if it is missing or stale (the C++ sources live next to this file).  There is no
pure-Python fallback: the sampler, seqlocks, renderer and HTTP server exist only
in C++.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None


def load(rebuild: bool = True):
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None:
            from . import build

            if rebuild and os.environ.get("KGS_NO_BUILD") != "1":
                build.build_native()
            _mod = importlib.import_module("kube_gpu_stats_amd._kgs_native")
    return _mod


def pmc_lib_path(source: str = "rocprofiler") -> str:
    """In-tree counter reader for a --pmc source: aqlprofile (direct) or rocprofiler."""
    from . import build

    return build.pmc_aql_lib_path() if source == "aqlprofile" else build.pmc_lib_path()
