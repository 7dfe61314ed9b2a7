#!/bin/bash
# Identify the thread that spins once rocprofiler device counting is initialised.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GPUID=$(KGS_NO_BUILD=1 python -c "from kube_gpu_stats_amd import native; N = native.load(); print(N.Exporter({'backend': 'amdsmi', 'port': -1}).devices()[0]['kfd_gpu_id'])")
echo "gpu_id=$GPUID"
LIB=$PWD/kube_gpu_stats_amd/lib/libkgs_pmc.so
timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" > gpurun_out/r11_default.jsonl 2>gpurun_out/r11_default.err
echo "default rc=$?"
HSA_ENABLE_INTERRUPT=1 timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" > gpurun_out/r11_interrupt.jsonl 2>&1
echo "interrupt rc=$?"
