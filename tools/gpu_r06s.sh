#!/bin/bash
# Round 6, session S: A @ dP1 gathered inside the RC_ENC0 launch at d = 128 (C5) -- the
# parity tests, then the C5 step against the separate SpMM launch (debug bit 128 at plan
# creation) and the C2 step as before, alternating processes, and the C5 timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/st
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
run 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_configs.py \
  -k "enc0 or gcn0 or c5 or 128 or c2_size or window" > gpurun_out/s_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/s_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels "" --tag c5_gather >> gpurun_out/s_ab.jsonl 2>>gpurun_out/s_err.log || exit 1
  run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels "" --step-debug 128 --tag c5_spmm >> gpurun_out/s_ab.jsonl 2>>gpurun_out/s_err.log || exit 1
  run 200 python tools/ab_run.py --kernels "" --tag c2 >> gpurun_out/s_ab.jsonl 2>>gpurun_out/s_err.log || exit 1
done
grep -o '"tag": "[a-z0-9_ ]*", "step_ms": [0-9.]*' gpurun_out/s_ab.jsonl
run 200 rocprofv3 --kernel-trace -d gpurun_out/st/s_c5 -o run --output-format csv \
  -- python tools/prof_step.py --config C5 --graphs 1 --steps 4 --graph > gpurun_out/s_st_c5.log 2>&1 || exit 1
python tools/step_timeline.py gpurun_out/st/s_c5/run_kernel_trace.csv > gpurun_out/st/s_c5.timeline.txt
cat gpurun_out/st/s_c5.timeline.txt
