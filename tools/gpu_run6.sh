#!/bin/bash
# rocprofv3 kernel trace of the bench with an *attached* exporter (PMC tier on),
# started outside the profiler so its rocprofiler-sdk counting context is its own.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
timeout -k 10 600 python -m kube_gpu_stats_amd.cli exporter --listen 127.0.0.1:19555 --hz 1000 --pmc rocprofiler \
   --control-http --proc-every 100 --link-every 1000 > gpurun_out/r6_exporter.log 2>&1 &
EP=$!
sleep 8
head -c 600 gpurun_out/r6_exporter.log; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attach -o bench -- \
   python3 bench.py --steps 60 --warmup 3 --attach 127.0.0.1:19555 --out gpurun_out/r6_bench_attach.json > gpurun_out/r6_rocprof.log 2>&1
rc=$?
echo "rocprof rc=$rc"
kill $EP; wait $EP
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 60 python tools/rocprof_overhead.py gpurun_out/prof_attach --warmup 3 --steps 60 --out gpurun_out/r6_rocprof_overhead.md
tail -4 gpurun_out/r6_rocprof_overhead.md
