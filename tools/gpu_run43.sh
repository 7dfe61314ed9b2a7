#!/bin/bash
# Counter hand-over on hardware: GPU suite (STOP/re-START test), then a user profiler (rocprofv3 --pmc) running
# while a live 8 kHz exporter has released the counters, then the exporter takes them back.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r43
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r43/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/r43/${name}.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_handover 200 python -u -m pytest tests/test_gpu.py -k handover -x -v -s --timeout 120 --timeout-method thread
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread
timeout -k 10 300 python -m kube_gpu_stats_amd.cli exporter --listen 127.0.0.1:19557 --hz 8000 --pmc aqlprofile \
   --proc-every 800 --link-every 8000 > gpurun_out/r43/exporter.log 2>&1 &
EP=$!
sleep 8
curl -s 127.0.0.1:19557/metrics | grep -E "^kgs_pmc_(enabled|samples_total)" > gpurun_out/r43/m_before.txt
kill -USR1 $EP; sleep 1
curl -s 127.0.0.1:19557/metrics | grep -E "^kgs_pmc_(enabled|samples_total)" > gpurun_out/r43/m_released.txt
step rocprof_pmc 200 rocprofv3 --pmc SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r43/prof_pmc -o user -- \
   python3 -c "import torch; a=torch.randn(4096,4096,device='cuda'); [a@a for _ in range(20)]; torch.cuda.synchronize(); print('user profiler run ok')"
kill -USR2 $EP; sleep 2
curl -s 127.0.0.1:19557/metrics | grep -E "^kgs_pmc_(enabled|samples_total|releases_total)|^amdgpu_gpu_clock_effective" > gpurun_out/r43/m_after.txt
kill $EP; wait $EP
cat gpurun_out/r43/m_before.txt gpurun_out/r43/m_released.txt gpurun_out/r43/m_after.txt
find gpurun_out/r43/prof_pmc -name "*counter_collection*" | head -3
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r43/prof_pmc/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0]))) if f else []
tot = {}
for r in rows:
    tot[r.get("Counter_Name")] = tot.get(r.get("Counter_Name"), 0.0) + float(r.get("Counter_Value") or 0)
print("user profiler counters:", len(rows), "rows", tot)
PY
du -sh gpurun_out
