#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r4_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/r4_${name}.log" | cut -c1-600
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step bench 300 python bench.py --steps 60 --warmup 3 --out gpurun_out/r4_bench.json
step bench_pmfw_only 300 python bench.py --steps 60 --warmup 3 --hz 100 --pmc none --out gpurun_out/r4_bench_pmfw.json
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 60 --warmup 3 --out gpurun_out/r4_bench_rocprof.json
step overhead 60 python tools/rocprof_overhead.py gpurun_out/prof_bench --warmup 3 --steps 60 --out gpurun_out/r4_rocprof_overhead.md
