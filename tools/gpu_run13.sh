#!/bin/bash
# Staged bring-up of the aqlprofile counter reader.  Each stage only runs if the
# previous one succeeded: (1) build packets without submitting, (2) START + 1 kHz
# READs for 1 s from the probe, (3) full bench with --pmc aqlprofile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KGS_NO_BUILD=1
GPUID=$(python -c "from kube_gpu_stats_amd import native; N = native.load(); print(N.Exporter({'backend': 'amdsmi', 'port': -1}).devices()[0]['kfd_gpu_id'])")
LIB=$PWD/kube_gpu_stats_amd/lib/libkgs_pmc_aql.so
echo "gpu_id=$GPUID"
KGS_AQL_DRY=1 timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" > gpurun_out/r13_dry.jsonl 2>gpurun_out/r13_dry.err
echo "dry rc=$?"; cat gpurun_out/r13_dry.jsonl | tail -1 | cut -c1-300
grep -q '"error":"open: dry: events=[1-9]' gpurun_out/r13_dry.jsonl || { echo "stop: dry stage did not build packets"; exit 3; }
timeout -k 10 60 tools/build/pmc_threads "$LIB" "$GPUID" > gpurun_out/r13_live.jsonl 2>gpurun_out/r13_live.err
rc=$?; echo "live rc=$rc"; tail -2 gpurun_out/r13_live.jsonl | cut -c1-400
[ $rc -eq 0 ] || exit 4
grep -q '"errors":0' gpurun_out/r13_live.jsonl || { echo "stop: live reads reported errors"; exit 5; }
timeout -k 10 300 python bench.py --pmc aqlprofile --out gpurun_out/r13_bench_aql.json > gpurun_out/r13_bench_aql.log 2>&1
echo "bench rc=$?"; tail -1 gpurun_out/r13_bench_aql.log | cut -c1-200
