#!/usr/bin/env python3
"""Headline benchmark entry point (the driver's contract):

    python bench.py --gpus N --steps K --warmup W

The phases live in the ``bench/`` package (bench/__init__.py describes them); this
file only puts the repository on sys.path and runs ``bench.cli.main``.  With N > 1
and no torchrun environment it starts N ranks itself (bench/cli.py spawn_ranks).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
