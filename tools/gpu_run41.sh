#!/bin/bash
# READ packet fences: drop the system-scope *acquire* (cache invalidate before each READ) but keep the
# release (orders the signal after the results); with and without the in-IB L2 writeback (lean 2 / 3).
# The MFMA util column is the correctness check (≈91 % under the MFMA loop).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r41
export KGS_NO_BUILD=1
timeout -k 10 600 python -u tools/launch_overhead.py 8000:base:aqlprofile:2 8000:base:aqlprofile:2:fence=none,sys \
  8000:base:aqlprofile:3:fence=none,sys 8000:base:aqlprofile:3:fence=none,agent off 8000:base:aqlprofile:2 \
  8000:base:aqlprofile:2:fence=none,sys 8000:base:aqlprofile:3:fence=none,sys 8000:base:aqlprofile:2:fence=agent,sys \
  off > gpurun_out/r41/launch.log 2>&1
rc=$?; echo "launch rc=$rc"; cp gpurun_out/launch_overhead.json gpurun_out/r41/; exit $rc
