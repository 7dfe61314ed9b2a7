#!/bin/bash
# Round checkpoint + real-framework load: GPU suite, smoke(), default bench, bench --load train (PyTorch bf16
# decoder fwd+bwd+AdamW as the workload) x2, rocprofv3 kernel stats of the train bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r50
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r50/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/r50/${name}.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread
step smoke 200 python __graft_entry__.py smoke
step bench_8k 200 python bench.py --out gpurun_out/r50/bench_8k.json
step bench_train 300 python bench.py --load train --steps 30 --warmup 5 --out gpurun_out/r50/bench_train.json
step bench_train_b 300 python bench.py --load train --steps 30 --warmup 5 --out gpurun_out/r50/bench_train_b.json
step rocprof_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r50/prof -o bench -- \
   python3 bench.py --load train --steps 15 --warmup 3 --out gpurun_out/r50/bench_train_under_rocprof.json
rm -f gpurun_out/r50/prof/*kernel_trace.csv gpurun_out/r50/prof/*agent_info.csv; du -sh gpurun_out
