#!/bin/bash
# Same box, same load: exporter with the aqlprofile reader vs the rocprofiler reader.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r17_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/r17_${name}.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; tail -30 gpurun_out/bench_exporter_r0.log; exit $rc; fi
}
step bench_aql 300 python bench.py --pmc aqlprofile --out gpurun_out/r17_bench_aql.json
cp gpurun_out/bench_exporter_r0.log gpurun_out/r17_exporter_aql.log
step bench_rocprof 300 python bench.py --pmc rocprofiler --out gpurun_out/r17_bench_rocprof.json
