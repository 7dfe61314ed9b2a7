"""Flag/env configuration.

The reference hard-codes every constant (Prometheus URL and proxy,
gpu_util_stats.py:9-12; namespace ``ava`` :133; step 3600 :137,155; window one
day :156; HTTP timeout 5 s :24,32; GPU resource name who_use_gpu.py:40; the
kubectl command who_use_gpu.py:8).  Here each one is a flag whose default can
also come from a ``KGS_<NAME>`` environment variable, and whose ``--compat``
default is the reference value.
"""
from __future__ import annotations

import argparse
import os
from typing import Any

ENV_PREFIX = "KGS_"

# Reference constants (compat defaults).
REF_PROM_URL = "http://prometheus.ke-xs-sys.qiniu.io/api/v1"  # gpu_util_stats.py:9
REF_PROXY = "http://10.34.33.80"                               # gpu_util_stats.py:11
REF_NAMESPACE = "ava"                                          # gpu_util_stats.py:133
REF_STEP_S = 3600                                              # gpu_util_stats.py:137,155
REF_WINDOW_S = 86400                                           # gpu_util_stats.py:156
REF_TIMEOUT_S = 5.0                                            # gpu_util_stats.py:24,32,107,119
REF_GPU_RESOURCE = "alpha.kubernetes.io/nvidia-gpu"            # who_use_gpu.py:40
REF_KUBECTL = "kubectl get pods --all-namespaces -o json"      # who_use_gpu.py:8

AMD_GPU_RESOURCE = "amd.com/gpu"


def env_default(name: str, default: Any) -> Any:
    """Value of KGS_<NAME> coerced to the type of ``default``; ``default`` if unset."""
    raw = os.environ.get(ENV_PREFIX + name.upper().replace("-", "_"))
    if raw is None:
        return default
    if isinstance(default, bool):
        return raw.strip().lower() in ("1", "true", "yes", "on")
    if isinstance(default, int):
        return int(raw)
    if isinstance(default, float):
        return float(raw)
    if isinstance(default, list):
        return [x for x in raw.split(",") if x]
    return raw


def add_flag(ap: argparse.ArgumentParser, name: str, default: Any, help: str, **kw) -> None:
    """``--name`` with an env override and the default shown in --help."""
    dflt = env_default(name, default)
    dest = name.replace("-", "_")
    if isinstance(default, bool):
        ap.add_argument(f"--{name}", dest=dest, default=dflt, action=argparse.BooleanOptionalAction,
                        help=f"{help} (env {ENV_PREFIX}{dest.upper()}; default {dflt})", **kw)
    else:
        typ = type(default) if default is not None and not isinstance(default, list) else str
        ap.add_argument(f"--{name}", dest=dest, default=dflt, type=typ,
                        help=f"{help} (env {ENV_PREFIX}{dest.upper()}; default {dflt})", **kw)
