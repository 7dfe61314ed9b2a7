#!/bin/bash
# Lean READ default + dispatch-bound bench component: GPU suite, bench 8 kHz lean 2 vs 0, 1 kHz, rocprof attached.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r33
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r33/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/r33/${name}.log" | cut -c1-250
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread
step bench_8k 200 python bench.py --out gpurun_out/r33/bench_8k.json
step bench_8k_lean0 200 python bench.py --pmc-lean 0 --out gpurun_out/r33/bench_8k_lean0.json
step bench_1k 200 python bench.py --hz 1000 --out gpurun_out/r33/bench_1k.json
step bench_8k_b 200 python bench.py --out gpurun_out/r33/bench_8k_b.json
timeout -k 10 300 python -m kube_gpu_stats_amd.cli exporter --listen 127.0.0.1:19555 --hz 8000 --pmc aqlprofile \
   --control-http --proc-every 800 --link-every 8000 > gpurun_out/r33/attached_exporter.log 2>&1 &
EP=$!
sleep 8
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r33/prof_attach -o bench -- \
   python3 bench.py --steps 60 --warmup 3 --attach 127.0.0.1:19555 --out gpurun_out/r33/bench_attach.json
kill $EP; wait $EP
step overhead 60 python tools/rocprof_overhead.py gpurun_out/r33/prof_attach --warmup 3 --steps 60 --out gpurun_out/r33/rocprof_overhead_8khz.md
rm -f gpurun_out/r33/prof_attach/*kernel_trace.csv gpurun_out/r33/prof_attach/*agent_info.csv; du -sh gpurun_out
