#!/bin/bash
# Fresh-container re-check: full GPU suite, smoke(), default bench, rocprofv3 kernel stats of the bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r20_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/r20_${name}.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 120 python __graft_entry__.py smoke
step bench 300 python bench.py --out gpurun_out/r20_bench.json
