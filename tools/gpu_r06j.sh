#!/bin/bash
# Round 6, session J: the decoder's backward and the backward head in one launch
# (dec_bwd_head_kernel) -- its bitwise test and the C2 tests, then the step and the
# kernels against the two separate launches (host bit 1 << 20), alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
run 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_c2_bench.py \
  -k "one_launch or fused or c2 or train_steps or window" > gpurun_out/j_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/j_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  run 200 python tools/ab_run.py --kernels dec:bwdhead,dec:bwd,head_bwd --tag fused >> gpurun_out/j_ab.jsonl 2>>gpurun_out/j_err.log || exit 1
  run 200 python tools/ab_run.py --kernels dec:bwd,head_bwd --tag apart --step-debug 1048576 >> gpurun_out/j_ab.jsonl 2>>gpurun_out/j_err.log || exit 1
done
cat gpurun_out/j_ab.jsonl
run 200 rocprofv3 --kernel-trace -d gpurun_out/st/j_g8 -o run --output-format csv \
  -- python tools/prof_step.py --graphs 8 --steps 6 --graph > gpurun_out/j_st_g8.log 2>&1 || exit 1
python tools/step_timeline.py gpurun_out/st/j_g8/run_kernel_trace.csv > gpurun_out/st/j_g8.timeline.txt
cat gpurun_out/st/j_g8.timeline.txt
