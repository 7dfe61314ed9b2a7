#!/bin/bash
# Per-XCD vector-memory (TA) busy: XCC-gated triad on XCDs {1, 6} under a --pmc-set full exporter; GPU suite.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r49
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r49/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/r49/${name}.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_xcd 200 python -u -m pytest tests/test_gpu.py -k xcd -x -v -s --timeout 120 --timeout-method thread
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread
grep -h "vmem_busy_xcc\|mfma_util_xcc" gpurun_out/r49/pytest_xcd.log | cut -c1-400
