#!/bin/bash
# Round 6, session D: why zzT reads ~11 us longer inside the step than back to back --
# a kernel trace of the captured C2 step with zzT launched twice (debug bit 1 << 17), and
# per-kernel effective clocks (GRBM_GUI_ACTIVE / GRBM_COUNT over the replays); the window
# SpMM's phase skips on the 256-graph batch (where its time goes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
run 200 rocprofv3 --kernel-trace -d gpurun_out/st/g8z2 -o run --output-format csv \
  -- python tools/prof_step.py --graphs 8 --steps 6 --graph --debug 131072 > gpurun_out/st_g8z2.log 2>&1
python tools/step_timeline.py gpurun_out/st/g8z2/run_kernel_trace.csv | tee gpurun_out/st/g8z2.timeline.txt
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_clk -o run --output-format csv \
  -- python tools/prof_step.py --graphs 8 --steps 3 --graph > gpurun_out/pmc_clk.log 2>&1
echo "pmc rc=$?"; ls gpurun_out/pmc_clk 2>/dev/null | head
run 300 python -u tools/ab_spmm_win.py --flags 0,16777216,33554432,67108864,100663296 --rounds 3 > gpurun_out/spmm_skips.txt 2>&1
echo "spmm rc=$?"; tail -12 gpurun_out/spmm_skips.txt
