#!/bin/bash
# Backtrace of the spinning HSA thread + mitigation experiments (MWAITX, SCHED_IDLE).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GPUID=$(KGS_NO_BUILD=1 python -c "from kube_gpu_stats_amd import native; N = native.load(); print(N.Exporter({'backend': 'amdsmi', 'port': -1}).devices()[0]['kfd_gpu_id'])")
LIB=$PWD/kube_gpu_stats_amd/lib/libkgs_pmc.so
timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" > gpurun_out/r12_bt.jsonl 2>gpurun_out/r12_bt.err
echo "bt rc=$?"
HSA_ENABLE_MWAITX=1 timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" > gpurun_out/r12_mwaitx.jsonl 2>gpurun_out/r12_mwaitx.err
echo "mwaitx rc=$?"
KGS_PROBE_SCHED_IDLE=1 timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" > gpurun_out/r12_idle.jsonl 2>gpurun_out/r12_idle.err
echo "idle rc=$?"
