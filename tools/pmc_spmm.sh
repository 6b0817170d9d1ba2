#!/bin/bash
# HBM traffic of the window SpMM on bench.py's 256-graph batch: one rocprofv3 --pmc pass per
# counter (FETCH_SIZE, WRITE_SIZE), summarised by tools/pmc_spmm_win.py.
#   bash tools/pmc_spmm.sh OUT_JSON
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=${1:-gpurun_out/pmc_spmm_win.json}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_spmm_fetch -o run --output-format csv \
  -- python tools/ab_spmm_win.py --flags 0 --rounds 1 > gpurun_out/pmc_spmm_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_spmm_write -o run --output-format csv \
  -- python tools/ab_spmm_win.py --flags 0 --rounds 1 > gpurun_out/pmc_spmm_write.log 2>&1 || exit $?
beta=$(grep -o "beta [0-9]*" gpurun_out/pmc_spmm_fetch.log | head -1 | cut -d' ' -f2)
nnz=$(grep -o "nnz [0-9]*" gpurun_out/pmc_spmm_fetch.log | head -1 | cut -d' ' -f2)
python tools/pmc_spmm_win.py gpurun_out/pmc_spmm_fetch gpurun_out/pmc_spmm_write "$out" --nnz $nnz --beta $beta
