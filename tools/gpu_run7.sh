#!/bin/bash
# Round-1 measurement sweep for BASELINE.md: gpu tests, smoke, bench at the config tiers.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r7_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/r7_${name}.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step pytest_gpu 400 python -m pytest tests/test_gpu.py -q -s
step smoke 120 python __graft_entry__.py smoke
step b1hz 300 python bench.py --steps 60 --warmup 3 --hz 1 --pmc none --out gpurun_out/r7_b1hz.json
step b10hz 300 python bench.py --steps 60 --warmup 3 --hz 10 --pmc none --out gpurun_out/r7_b10hz.json
step b100hz 300 python bench.py --steps 60 --warmup 3 --hz 100 --out gpurun_out/r7_b100hz.json
step b1khz 300 python bench.py --steps 60 --warmup 3 --out gpurun_out/r7_b1khz.json
step b2khz 300 python bench.py --steps 60 --warmup 3 --hz 2000 --out gpurun_out/r7_b2khz.json
