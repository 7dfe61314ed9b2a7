#!/bin/bash
# Launch-bound interference, repeated: is r37's 8 kHz graph slowdown real, and is it the READs, the
# per-process tier or the 1 µs timer slack?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r38
export KGS_NO_BUILD=1
timeout -k 10 500 python -u tools/launch_overhead.py 8000:base:aqlprofile:2 8000:base:aqlprofile:2:proc=0 \
  8000:base:aqlprofile:2:slack=50000 off 8000:base:aqlprofile:2 8000:base:none:2 1000:base:aqlprofile:2 off \
  8000:base:aqlprofile:2:proc=0 > gpurun_out/r38/launch.log 2>&1
rc=$?; echo "launch rc=$rc"; tail -12 gpurun_out/r38/launch.log | cut -c1-60,200-400; cp gpurun_out/launch_overhead.json gpurun_out/r38/; exit $rc
