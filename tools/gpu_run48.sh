#!/bin/bash
# rocprofv3 --pmc profile of the hand-written load kernels: MFMA MOPs / MfmaUtil, HBM FETCH / WRITE sizes vs the
# known work of each kernel.  One counter pass per run (TCC: FETCH_SIZE uses 3 counters, WRITE_SIZE 2).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r48
export KGS_NO_BUILD=1
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/r48/$name -o k -- python3 tools/pmc_kernels.py \
     > gpurun_out/r48/$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
timeout -k 10 120 python3 tools/pmc_kernels.py > gpurun_out/r48/work.log 2>&1 || exit 1
pass sq SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE MfmaUtil
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 tools/pmc_kernels_report.py gpurun_out/r48 | tee gpurun_out/r48/report.md
find gpurun_out/r48 -name "*agent_info.csv" -delete; du -sh gpurun_out
