#!/bin/bash
# Per-XCD counter placement: XCC-gated test with the reader's raw result dump.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r36
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r36/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/r36/${name}.log" | cut -c1-250
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_xcd 200 python -u -m pytest tests/test_gpu.py -k xcd -x -v -s --timeout 120 --timeout-method thread
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread
step smoke 200 python __graft_entry__.py smoke
step bench_8k 200 python bench.py --out gpurun_out/r36/bench_8k.json
du -sh gpurun_out
