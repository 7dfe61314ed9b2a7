#!/bin/bash
# Exporter CPU cost on hardware: per-thread breakdown with and without the PMC tier.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r10_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/r10_${name}.log" | cut -c1-200
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step bench_1k 300 python bench.py --out gpurun_out/r10_bench_1k.json
step bench_nopmc 300 python bench.py --pmc none --out gpurun_out/r10_bench_nopmc.json
step bench_100 300 python bench.py --hz 100 --out gpurun_out/r10_bench_100.json
