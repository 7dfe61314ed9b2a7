#!/bin/bash
# Where does the +0.2-0.3 % on the PyTorch training load (r50) come from?  Train bench, 60 steps per phase:
# 8 kHz (default) / 1 kHz / PMFW only at 100 Hz (no counter READs) / 8 kHz with no /metrics scrapes
# during phase B (the scraper is a thread of the bench process and competes for its GIL).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r51
export KGS_NO_BUILD=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/r51/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/r51/${name}.log" | cut -c1-160
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
T="python bench.py --load train --steps 60 --warmup 5"
step train_8k 240 $T --out gpurun_out/r51/train_8k.json
step train_1k 240 $T --hz 1000 --out gpurun_out/r51/train_1k.json
step train_pmfw100 240 $T --hz 100 --pmc none --out gpurun_out/r51/train_pmfw100.json
step train_8k_noscrape 240 $T --scrape-hz 0.001 --out gpurun_out/r51/train_8k_noscrape.json
step train_8k_b 240 $T --out gpurun_out/r51/train_8k_b.json
