#!/bin/bash
mkdir -p gpurun_out
export KGS_NO_BUILD=1
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r2_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/r2_${name}.log" | cut -c1-1500
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step pmc_probe 300 python tools/pmc_probe_run.py
step pmc_debug 240 python tools/pmc_debug.py
step bench 300 python bench.py --steps 40 --warmup 3 --out gpurun_out/r2_bench.json
