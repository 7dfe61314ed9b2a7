#!/bin/bash
# aqlprofile reader with the exporter's 4-counter set: probe first, then the exporter itself.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1 PYTHONFAULTHANDLER=1
GPUID=$(python -c "from kube_gpu_stats_amd import native; N = native.load(); print(N.Exporter({'backend': 'amdsmi', 'port': -1}).devices()[0]['kfd_gpu_id'])")
LIB=$PWD/kube_gpu_stats_amd/lib/libkgs_pmc_aql.so
KGS_AQL_DRY=1 timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" GRBM_COUNT:max GRBM_GUI_ACTIVE:max SQ_VALU_MFMA_BUSY_CYCLES TA_TA_BUSY:mean > gpurun_out/r14_dry4.jsonl 2>&1
echo "dry4 rc=$?"; tail -1 gpurun_out/r14_dry4.jsonl | cut -c1-300
timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" GRBM_COUNT:max GRBM_GUI_ACTIVE:max SQ_VALU_MFMA_BUSY_CYCLES TA_TA_BUSY:mean > gpurun_out/r14_live4.jsonl 2>gpurun_out/r14_live4.err
rc=$?; echo "live4 rc=$rc"; tail -1 gpurun_out/r14_live4.jsonl | cut -c1-400; tail -5 gpurun_out/r14_live4.err
[ $rc -eq 0 ] || exit 4
timeout -k 10 -s INT 10 python -m kube_gpu_stats_amd.cli exporter --listen 127.0.0.1:0 --hz 100 --pmc aqlprofile > gpurun_out/r14_exporter.out 2> gpurun_out/r14_exporter.err
echo "exporter rc=$?"; head -c 1500 gpurun_out/r14_exporter.out; echo; tail -30 gpurun_out/r14_exporter.err
