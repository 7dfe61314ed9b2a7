#!/bin/bash
# Lean READ experiment: launch-bound interference + counter sanity per READ variant.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r31
export KGS_NO_BUILD=1
timeout -k 10 500 python -u tools/launch_overhead.py 1000:base:aqlprofile:0 1000:base:aqlprofile:1 \
   1000:base:aqlprofile:2 1000:base:aqlprofile:3 8000:base:aqlprofile:0 8000:base:aqlprofile:2 \
   8000:base:aqlprofile:3 1000:full:aqlprofile:2 > gpurun_out/r31/launch.log 2>&1
rc=$?; echo "launch rc=$rc"; tail -12 gpurun_out/r31/launch.log; cp gpurun_out/launch_overhead.json gpurun_out/r31/; exit $rc
