#!/bin/bash
# Counter probe through the direct aqlprofile reader: TCC (HBM bytes), SQ, TCP under known loads.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
timeout -k 10 240 python -u tools/aql_probe.py > gpurun_out/r21_aql_probe.log 2>&1
rc=$?; echo "rc=$rc"; tail -c 3000 gpurun_out/r21_aql_probe.log; exit $rc
