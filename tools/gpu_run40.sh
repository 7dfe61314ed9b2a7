#!/bin/bash
# Cheaper READs?  AQL header fences (sys/agent/none) and poll-only completion signals, 8 kHz, launch-bound graph;
# counter sanity (MFMA util under an MFMA loop) is printed per phase.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r40
export KGS_NO_BUILD=1
timeout -k 10 600 python -u tools/launch_overhead.py 8000:base:aqlprofile:2 8000:base:aqlprofile:2:fence=none \
  8000:base:aqlprofile:2:signal=poll 8000:base:aqlprofile:2:fence=none:signal=poll off \
  8000:base:aqlprofile:2:fence=agent 8000:base:aqlprofile:2 8000:base:aqlprofile:2:fence=none:signal=poll \
  8000:base:aqlprofile:3:fence=none:signal=poll off > gpurun_out/r40/launch.log 2>&1
rc=$?; echo "launch rc=$rc"; tail -12 gpurun_out/r40/launch.log | cut -c1-70,200-330; cp gpurun_out/launch_overhead.json gpurun_out/r40/; exit $rc
