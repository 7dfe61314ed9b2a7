#!/bin/bash
# Round checkpoint of the current tree: GPU suite, smoke(), default bench ×2, rocprofv3 kernel stats of the bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r47
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r47/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/r47/${name}.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread
step smoke 200 python __graft_entry__.py smoke
step bench_8k 200 python bench.py --out gpurun_out/r47/bench_8k.json
step bench_8k_b 200 python bench.py --out gpurun_out/r47/bench_8k_b.json
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r47/prof -o bench -- \
   python3 bench.py --steps 40 --warmup 3 --out gpurun_out/r47/bench_under_rocprof.json
rm -f gpurun_out/r47/prof/*kernel_trace.csv gpurun_out/r47/prof/*agent_info.csv; du -sh gpurun_out
