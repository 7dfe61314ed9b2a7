#!/bin/bash
# First-exporter effect on a launch-bound HIP graph: trace it for 20 s on a fresh box, then the A/B set again.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r39
export KGS_NO_BUILD=1
KGS_FIRST_TRACE=20 timeout -k 10 500 python -u tools/launch_overhead.py 8000:base:aqlprofile:2 8000:base:aqlprofile:2:proc=0 \
  off 8000:base:aqlprofile:2 1000:base:aqlprofile:2 16000:base:aqlprofile:2 > gpurun_out/r39/launch.log 2>&1
rc=$?; echo "launch rc=$rc"; grep first_exporter gpurun_out/r39/launch.log | cut -c1-1500; tail -8 gpurun_out/r39/launch.log | cut -c1-60,200-400; cp gpurun_out/launch_overhead.json gpurun_out/r39/; exit $rc
