#!/bin/bash
# rocprofv3 kernel trace of bench.py, split by exporter condition.  The exporter
# runs OUTSIDE the profiler (its private AQL queue and HSA client must not be
# intercepted) and the bench drives it over --attach; A/C are then "paused", not
# "absent".  The multi-100-MB trace CSV is reduced to a summary on the box and
# deleted.   usage: bash tools/gpu_rocprof.sh <outdir>
set -u
OUT=${1:-gpurun_out/rocprof}
mkdir -p "$OUT"
export TMPDIR=/tmp
BDF=$(python3 -c "import torch;p=torch.cuda.get_device_properties(0);print(f'{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0')")
python3 -m kube_gpu_stats_amd.cli exporter --listen 127.0.0.1:19400 --hz 8000 --pmc aqlprofile --control-http \
  --proc-period 0.1 --link-period 1 --window 2 --bdfs "$BDF" --node-name rocprof-node > "$OUT/exporter.out" 2> "$OUT/exporter.err" &
EXP=$!
for i in $(seq 60); do grep -q '"event": "ready"' "$OUT/exporter.out" 2>/dev/null && break; sleep 1; done
if ! grep -q '"event": "ready"' "$OUT/exporter.out"; then echo "exporter not ready"; kill $EXP; exit 1; fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py --steps 6 --warmup 2 \
  --step-ms ${KGS_ROCPROF_STEP_MS:-450} --rounds 24 --util-s 0 --idle-power-s 0 --released 0 --attach 127.0.0.1:19400 --out "$OUT/bench_rocprof.json" > "$OUT/bench.log" 2>&1
RC=$?
kill $EXP; wait $EXP 2>/dev/null
echo "rocprof rc=$RC"
if [ $RC -ne 0 ]; then tail -20 "$OUT/bench.log"; exit $RC; fi
python3 tools/rocprof_overhead.py "$OUT/trace" "$OUT/bench_rocprof.json" --out "$OUT/rocprof_overhead.md" > "$OUT/split.json"
RC=$?
# keep only the per-kernel statistics: the trace itself is hundreds of MB, and
# gpurun copies nothing back once gpurun_out/ passes 64 MiB
find "$OUT/trace" -type f ! -name '*stats.csv' -delete
cat "$OUT/rocprof_overhead.md"
exit $RC
