#!/bin/bash
# rocprofv3 passes over tools/prof_spmm.py: register-gather vs row-tiled bf16 SpMM
# on the 256-graph batch (kernel trace), then SQ / TCC counters of the tiled kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pt
run() {  # run NAME ROCPROF-ARGS... -- SCRIPT-ARGS...
  local n=$1; shift
  timeout -k 5 90 rocprofv3 "$@" > gpurun_out/pt/$n.log 2>&1 || { echo "FAILED $n"; exit 1; }
}
KT="--kernel-trace --stats --output-format csv"
run kt_reg $KT -d gpurun_out/pt/kt_reg -o run -- python tools/prof_spmm.py --reps 10
run kt_t128 $KT -d gpurun_out/pt/kt_t128 -o run -- python tools/prof_spmm.py --reps 10 --tile-rows 128
run kt_t32 $KT -d gpurun_out/pt/kt_t32 -o run -- python tools/prof_spmm.py --reps 10 --tile-rows 32
run kt_t64 $KT -d gpurun_out/pt/kt_t64 -o run -- python tools/prof_spmm.py --reps 10 --tile-rows 64
run sq_t64 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pt/sq_t64 -o run -- python tools/prof_spmm.py --reps 3 --tile-rows 64
run fetch_t64 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pt/fetch_t64 -o run -- python tools/prof_spmm.py --reps 3 --tile-rows 64
run write_t64 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pt/write_t64 -o run -- python tools/prof_spmm.py --reps 3 --tile-rows 64
echo done
