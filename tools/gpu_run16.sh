#!/bin/bash
# aqlprofile reader, exporter counter set: dry (packet build only) -> live probe.  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
GPUID=$(python -c "from kube_gpu_stats_amd import native; N = native.load(); print(N.Exporter({'backend': 'amdsmi', 'port': -1}).devices()[0]['kfd_gpu_id'])")
LIB=$PWD/kube_gpu_stats_amd/lib/libkgs_pmc_aql.so
SET="GRBM_COUNT:max GRBM_GUI_ACTIVE:max SQ_VALU_MFMA_BUSY_CYCLES TA_TA_BUSY:mean"
KGS_AQL_DEBUG=1 KGS_AQL_DRY=1 timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" $SET > gpurun_out/r16_dry.jsonl 2> gpurun_out/r16_dry.err
rc=$?; echo "dry rc=$rc"; tail -1 gpurun_out/r16_dry.jsonl | cut -c1-200; cat gpurun_out/r16_dry.err | head -30
[ $rc -eq 1 ] || { echo "stop: dry stage rc=$rc"; exit 3; }
grep -q '"error":"open: dry: events=' gpurun_out/r16_dry.jsonl || { echo "stop: no packets"; exit 3; }
KGS_AQL_DEBUG=1 timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" $SET > gpurun_out/r16_live.jsonl 2> gpurun_out/r16_live.err
rc=$?; echo "live rc=$rc"; tail -1 gpurun_out/r16_live.jsonl | cut -c1-400; tail -12 gpurun_out/r16_live.err
exit $rc
