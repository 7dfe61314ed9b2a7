#!/bin/bash
# Rate sweep with lean READs, timer slack 1 µs and one catch-up tick: bench at 8/12/16/24 kHz, launch-bound probe.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r37
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r37/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/r37/${name}.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step bench_8k 200 python bench.py --out gpurun_out/r37/bench_8k.json
step bench_12k 200 python bench.py --hz 12000 --out gpurun_out/r37/bench_12k.json
step bench_16k 200 python bench.py --hz 16000 --out gpurun_out/r37/bench_16k.json
step bench_24k 200 python bench.py --hz 24000 --out gpurun_out/r37/bench_24k.json
step launch 400 python -u tools/launch_overhead.py 8000:base:aqlprofile:2 16000:base:aqlprofile:2 24000:base:aqlprofile:2
cp gpurun_out/launch_overhead.json gpurun_out/r37/ 2>/dev/null
du -sh gpurun_out
