"""Logging to stderr; stdout stays clean for reports."""
from __future__ import annotations

import logging
import os
import sys

_configured = False


def get(name: str = "kgs") -> logging.Logger:
    global _configured
    if not _configured:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
        root = logging.getLogger("kgs")
        root.addHandler(h)
        root.setLevel(os.environ.get("KGS_LOG_LEVEL", "INFO").upper())
        root.propagate = False
        _configured = True
    return logging.getLogger(name if name.startswith("kgs") else "kgs." + name)
