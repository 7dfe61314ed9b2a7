#!/bin/bash
mkdir -p gpurun_out
export KGS_NO_BUILD=1
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r3_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/r3_${name}.log" | cut -c1-800
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step pytest_gpu 400 python -m pytest tests/test_gpu.py -q -s
step bench100 300 python bench.py --steps 60 --warmup 3 --hz 100 --out gpurun_out/r3_bench100.json
step bench500 300 python bench.py --steps 60 --warmup 3 --hz 500 --out gpurun_out/r3_bench500.json
step bench1000 300 python bench.py --steps 60 --warmup 3 --hz 1000 --out gpurun_out/r3_bench1000.json
step bench2000 300 python bench.py --steps 60 --warmup 3 --hz 2000 --out gpurun_out/r3_bench2000.json
