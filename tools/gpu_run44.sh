#!/bin/bash
# Does a live exporter disturb a user's rocprofv3 --pmc run, and does the hand-over help?  Same user workload
# (20 fp32 4096² matmuls) profiled: (C) no exporter, (A) 8 kHz exporter holding the counters, (B) exporter
# released by SIGUSR1; then SIGUSR2 and the exporter's own counters are checked under an MFMA load.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r44
export KGS_NO_BUILD=1
USER_CMD='import torch; a=torch.randn(4096,4096,device="cuda"); [a@a for _ in range(20)]; torch.cuda.synchronize(); print("user profiler run ok")'
prof() {  # $1 = tag
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r44/prof_$1 -o user \
     -- python3 -c "$USER_CMD" > gpurun_out/r44/prof_$1.log 2>&1
  local rc=$?; echo "== prof_$1 rc=$rc"; return $rc
}
metrics() { curl -s 127.0.0.1:19558/metrics | grep -E "^kgs_pmc_(enabled|samples_total|releases_total)|^amdgpu_gpu_clock_effective|^amdgpu_mfma_util_percent" > gpurun_out/r44/m_$1.txt; }
prof C || exit 1
timeout -k 10 400 python -m kube_gpu_stats_amd.cli exporter --listen 127.0.0.1:19558 --hz 8000 --pmc aqlprofile \
   --proc-every 800 --link-every 8000 > gpurun_out/r44/exporter.log 2>&1 &
TP=$!
sleep 8
EP=$(pgrep -P $TP)   # the exporter itself (child of timeout): signals go to it, not to timeout
echo "exporter pid $EP"
metrics start
prof A || { kill $EP; exit 1; }
metrics after_A
kill -USR1 $EP; sleep 1
metrics released
prof B || { kill $EP; exit 1; }
kill -USR2 $EP; sleep 1
timeout -k 10 60 python3 -c "
import time, torch, sys
sys.path.insert(0, '.')
from kube_gpu_stats_amd.ops.load import LoadStep
ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=1 << 28)
t0 = time.time()
while time.time() - t0 < 2.0:
    ls.run_mfma(); torch.cuda.synchronize()
print('mfma load done')" > gpurun_out/r44/mfma_load.log 2>&1
metrics after_B
kill $EP; wait $TP
for t in start after_A released after_B; do echo "-- $t"; cat gpurun_out/r44/m_$t.txt; done
python3 - <<'PY'
import csv, glob
for tag in "CAB":
    f = glob.glob(f"gpurun_out/r44/prof_{tag}/**/*counter_collection.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0]))) if f else []
    tot = {}
    for r in rows:
        tot[r.get("Counter_Name")] = tot.get(r.get("Counter_Name"), 0.0) + float(r.get("Counter_Value") or 0)
    print(tag, len(rows), "rows", {k: int(v) for k, v in sorted(tot.items())})
PY
rm -rf gpurun_out/r44/prof_*/*agent_info.csv; du -sh gpurun_out
