#!/bin/bash
# Round 6, session H (round-end evidence, part 2): the headline bench under rocprofv3
# --kernel-trace --stats, the C2 step's per-kernel HBM traffic (FETCH / WRITE passes), the
# window SpMM's traffic on the 256-graph batch, the C2 step timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STAGES="profh traffic timeline" TAILN=8 bash tools/gpu_session.sh || exit $?
timeout -k 10 300 bash tools/pmc_spmm.sh gpurun_out/r06_pmc_spmm_win.json > gpurun_out/pmc_spmm.log 2>&1
echo "pmc_spmm rc=$?"; tail -20 gpurun_out/pmc_spmm.log
