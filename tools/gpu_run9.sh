#!/bin/bash
# GPU tests on the recovery-enabled backend + default bench + PMC rate sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r9_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/r9_${name}.log" | cut -c1-300
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step pytest_gpu 400 python -m pytest tests/test_gpu.py -q -s
step bench_1k 300 python bench.py --out gpurun_out/r9_bench_1k.json
step bench_2k 300 python bench.py --hz 2000 --out gpurun_out/r9_bench_2k.json
step bench_4k 300 python bench.py --hz 4000 --out gpurun_out/r9_bench_4k.json
step bench_8k 300 python bench.py --hz 8000 --out gpurun_out/r9_bench_8k.json
