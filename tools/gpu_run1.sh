#!/bin/bash
# Hardware pass: diagnostics, gpu tests, smoke, bench.  Each GPU step has its own time limit;
# a test failure (rc 1) does not stop the script, a timeout / signal (rc >= 124) does.
mkdir -p gpurun_out
export KGS_NO_BUILD=1
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r1_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/r1_${name}.log"
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step pmc_debug 240 python tools/pmc_debug.py
step pytest_gpu 400 python -m pytest tests/test_gpu.py -q -s
step smoke 120 python __graft_entry__.py smoke
step bench 300 python bench.py --steps 40 --warmup 3 --out gpurun_out/r1_bench.json
