#!/bin/bash
# Faster render + lean scrape client: GPU suite, smoke, bench default (8 kHz) x2, 100 Hz, 1 Hz PMFW-only.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r24
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r24/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/r24/${name}.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread
step smoke 120 python __graft_entry__.py smoke
step bench_default 200 python bench.py --out gpurun_out/r24/bench_default.json
step bench_default2 200 python bench.py --out gpurun_out/r24/bench_default2.json
step bench_100hz 200 python bench.py --hz 100 --out gpurun_out/r24/bench_100hz.json
step bench_1hz_nopmc 200 python bench.py --hz 1 --pmc none --out gpurun_out/r24/bench_1hz_nopmc.json
