#!/bin/bash
# Pipelined aqlprofile READs: counter-reader GPU tests (pipelined / sync / rocprofiler) + rate sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r22
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r22/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/r22/${name}.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_pmc 300 python -u -m pytest tests/test_gpu.py -k counter_reader -x -v -s --timeout 120 --timeout-method thread
step bench_1k_pipe 200 python bench.py --hz 1000 --out gpurun_out/r22/bench_1k_pipe.json
step bench_1k_sync 200 python bench.py --hz 1000 --pmc-pipeline 0 --out gpurun_out/r22/bench_1k_sync.json
step bench_4k_pipe 200 python bench.py --hz 4000 --out gpurun_out/r22/bench_4k_pipe.json
step bench_4k_sync 200 python bench.py --hz 4000 --pmc-pipeline 0 --out gpurun_out/r22/bench_4k_sync.json
step bench_8k_pipe 200 python bench.py --hz 8000 --out gpurun_out/r22/bench_8k_pipe.json
step bench_12k_pipe 200 python bench.py --hz 12000 --out gpurun_out/r22/bench_12k_pipe.json
