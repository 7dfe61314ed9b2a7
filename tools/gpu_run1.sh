#!/bin/bash
# First hardware pass: gpu tests, smoke, bench.  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export KGS_NO_BUILD=1
timeout -k 10 400 python -m pytest tests/test_gpu.py -x -q -s > gpurun_out/r1_pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -50 gpurun_out/r1_pytest_gpu.log; exit 1; }
tail -5 gpurun_out/r1_pytest_gpu.log
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/r1_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -30 gpurun_out/r1_smoke.log; exit 1; }
tail -2 gpurun_out/r1_smoke.log
timeout -k 10 300 python bench.py --steps 40 --warmup 3 --out gpurun_out/r1_bench.json > gpurun_out/r1_bench.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/r1_bench.log; exit 1; }
tail -1 gpurun_out/r1_bench.log
