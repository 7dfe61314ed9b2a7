#!/bin/bash
# Host-side crash hunt in the aqlprofile reader's open() (dry mode: no packet is ever submitted).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
GPUID=$(python -c "from kube_gpu_stats_amd import native; N = native.load(); print(N.Exporter({'backend': 'amdsmi', 'port': -1}).devices()[0]['kfd_gpu_id'])")
LIB=$PWD/kube_gpu_stats_amd/lib/libkgs_pmc_aql.so
for c in TA_TA_BUSY:mean SQ_VALU_MFMA_BUSY_CYCLES; do
  KGS_AQL_DEBUG=1 KGS_AQL_DRY=1 timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" GRBM_COUNT:max $c > gpurun_out/r15_$c.jsonl 2> gpurun_out/r15_$c.err
  echo "== $c rc=$?"; tail -1 gpurun_out/r15_$c.jsonl | cut -c1-200; cat gpurun_out/r15_$c.err | head -40
done
