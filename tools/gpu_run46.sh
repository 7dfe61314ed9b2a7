#!/bin/bash
# Periodic re-START (--pmc-refresh-s 5) after a user rocprofv3 --pmc run reprogrammed the counter selects (r45: MFMA 0 under load).
# (run r44 showed the clobbering); GPU suite and the default bench as regression checks.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r46
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r46/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/r46/${name}.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}


USER_CMD='import torch; a=torch.randn(4096,4096,device="cuda"); [a@a for _ in range(20)]; torch.cuda.synchronize(); print("user profiler run ok")'
metrics() { curl -s 127.0.0.1:19560/metrics | grep -E "^kgs_pmc_(enabled|stalled|reclaims_total|refreshes_total|samples_total)|^amdgpu_gpu_clock_effective|^amdgpu_mfma_util_percent" > gpurun_out/r46/m_$1.txt; }
timeout -k 10 300 python -m kube_gpu_stats_amd.cli exporter --listen 127.0.0.1:19560 --hz 8000 --pmc aqlprofile \
   --pmc-reclaim-s 5 --pmc-refresh-s 5 --proc-every 800 --link-every 8000 > gpurun_out/r46/exporter.log 2>&1 &
TP=$!
sleep 8
metrics start
step user_prof 200 rocprofv3 --pmc SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r46/prof_user -o user \
   -- python3 -c "$USER_CMD"
sleep 1; metrics after_user
sleep 6; metrics after_reclaim
timeout -k 10 60 python3 -c "
import time, torch, sys
sys.path.insert(0, '.')
from kube_gpu_stats_amd.ops.load import LoadStep
ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=1 << 28)
t0 = time.time()
while time.time() - t0 < 2.0:
    ls.run_mfma(); torch.cuda.synchronize()
import urllib.request
body = urllib.request.urlopen('http://127.0.0.1:19560/metrics', timeout=5).read().decode()
print([l for l in body.splitlines() if l.startswith(('amdgpu_mfma_util_percent', 'amdgpu_gpu_active_percent'))])
print('mfma load done')" > gpurun_out/r46/mfma_load.log 2>&1
metrics after_load
kill $(pgrep -P $TP); wait $TP
for t in start after_user after_reclaim after_load; do echo "-- $t"; cat gpurun_out/r46/m_$t.txt | sed 's/{gpu="0",uuid="[^"]*"}//'; done
cat gpurun_out/r46/mfma_load.log | cut -c1-300; rm -rf gpurun_out/r46/prof_user; du -sh gpurun_out
