#!/bin/bash
# Pipelined reader at the new 8 kHz bench default: GPU suite, smoke, bench (8 kHz and 100 Hz),
# rocprofv3 kernel trace of the bench with an attached 8 kHz exporter.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r23
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r23/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/r23/${name}.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread
step smoke 120 python __graft_entry__.py smoke
step bench_default 200 python bench.py --out gpurun_out/r23/bench_default.json
step bench_100hz 200 python bench.py --hz 100 --out gpurun_out/r23/bench_100hz.json
timeout -k 10 300 python -m kube_gpu_stats_amd.cli exporter --listen 127.0.0.1:19555 --hz 8000 --pmc aqlprofile \
   --control-http --proc-every 800 --link-every 8000 > gpurun_out/r23/attached_exporter.log 2>&1 &
EP=$!
sleep 8
head -c 400 gpurun_out/r23/attached_exporter.log; echo
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r23/prof_attach -o bench -- \
   python3 bench.py --steps 60 --warmup 3 --attach 127.0.0.1:19555 --out gpurun_out/r23/bench_attach.json
kill $EP; wait $EP
step overhead 60 python tools/rocprof_overhead.py gpurun_out/r23/prof_attach --warmup 3 --steps 60 --out gpurun_out/r23/rocprof_overhead_8khz.md
