# rocprofv3 passes over tools/prof_spmm.py (the bf16 SpMM on a 256-graph batch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ps
run() {  # run NAME ARGS... -- SCRIPT-ARGS...
  local n=$1; shift
  timeout -k 5 90 rocprofv3 "$@" > gpurun_out/ps/$n.log 2>&1 || { echo "FAILED $n"; exit 1; }
}
run kt_loc --kernel-trace --stats -d gpurun_out/ps/kt_loc -o run --output-format csv -- python tools/prof_spmm.py --reps 10
run kt_nat --kernel-trace --stats -d gpurun_out/ps/kt_nat -o run --output-format csv -- python tools/prof_spmm.py --reps 10 --no-locality
run hit_loc --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/ps/hit_loc -o run --output-format csv -- python tools/prof_spmm.py --reps 3
echo done
