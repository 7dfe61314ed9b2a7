#!/bin/bash
# Per-XCD counter placement: XCC-gated test with the reader's raw result dump (first run of the order placement).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r35
export KGS_NO_BUILD=1
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -k xcd -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r35/pytest_xcd.log 2>&1
