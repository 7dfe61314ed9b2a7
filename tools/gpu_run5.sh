#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r5_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/r5_${name}.log" | cut -c1-400
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step pytest_gpu 400 python -m pytest tests/test_gpu.py -q -s
step bench 300 python bench.py --steps 60 --warmup 3 --out gpurun_out/r5_bench.json
step bench2k 300 python bench.py --steps 60 --warmup 3 --hz 2000 --out gpurun_out/r5_bench2k.json
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench5 -o bench -- python3 bench.py --steps 60 --warmup 3 --out gpurun_out/r5_bench_rocprof.json
step overhead 60 python tools/rocprof_overhead.py gpurun_out/prof_bench5 --warmup 3 --steps 60 --out gpurun_out/r5_rocprof_overhead.md
