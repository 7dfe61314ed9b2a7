#!/bin/bash
# READ packet anatomy (PM4 dump) + launch-bound interference per counter set / rate.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r28
export KGS_NO_BUILD=1
for set in base full; do
  KGS_AQL_DUMP=1 KGS_AQL_DRY=1 timeout -k 10 60 python -m kube_gpu_stats_amd.cli exporter --listen 127.0.0.1:0 \
     --hz 10 --pmc aqlprofile --pmc-set $set --control-stdin < /dev/null > gpurun_out/r28/dump_$set.out 2> gpurun_out/r28/dump_$set.err
  echo "dump $set rc=$?"
done
timeout -k 10 400 python -u tools/launch_overhead.py > gpurun_out/r28/launch.log 2>&1
rc=$?; echo "launch rc=$rc"; tail -12 gpurun_out/r28/launch.log; exit $rc
