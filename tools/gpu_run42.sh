#!/bin/bash
# New default READ fences (acquire none, release system): GPU suite, bench ×2, launch-bound A/B vs the old fences,
# rocprofv3 kernel stats of the bench with an attached 8 kHz exporter.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r42
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r42/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/r42/${name}.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread
step bench_8k 200 python bench.py --out gpurun_out/r42/bench_8k.json
step bench_8k_b 200 python bench.py --out gpurun_out/r42/bench_8k_b.json
step launch 500 python -u tools/launch_overhead.py 8000:base:aqlprofile:2 8000:base:aqlprofile:2:fence=sys off \
   8000:base:aqlprofile:2 8000:base:aqlprofile:2:fence=sys 1000:base:aqlprofile:2
cp gpurun_out/launch_overhead.json gpurun_out/r42/
timeout -k 10 300 python -m kube_gpu_stats_amd.cli exporter --listen 127.0.0.1:19556 --hz 8000 --pmc aqlprofile \
   --control-http --proc-every 800 --link-every 8000 > gpurun_out/r42/attached_exporter.log 2>&1 &
EP=$!
sleep 8
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r42/prof_attach -o bench -- \
   python3 bench.py --steps 60 --warmup 3 --attach 127.0.0.1:19556 --out gpurun_out/r42/bench_attach.json
kill $EP; wait $EP
step overhead 60 python tools/rocprof_overhead.py gpurun_out/r42/prof_attach --warmup 3 --steps 60 --out gpurun_out/r42/rocprof_overhead_8khz.md
rm -f gpurun_out/r42/prof_attach/*kernel_trace.csv gpurun_out/r42/prof_attach/*agent_info.csv; du -sh gpurun_out
