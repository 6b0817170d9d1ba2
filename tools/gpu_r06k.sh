#!/bin/bash
# Round 6, session K: the fused decoder at d = 128 with streamed weights (C5) -- the fused
# decoder tests and the C5 / d = 128 config tests, then the C5 step and its kernels against
# the row-engine decoder (ab/c5base.so, the tree before), alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
run 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_configs.py \
  -k "fused_decoder or c5 or d128 or 128" > gpurun_out/k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/k_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels zzt_dense --tag c5fused >> gpurun_out/k_ab.jsonl 2>>gpurun_out/k_err.log || exit 1
  SND_LIB_PATH=ab/c5base.so run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels zzt_dense --tag c5rowengine >> gpurun_out/k_ab.jsonl 2>>gpurun_out/k_err.log || exit 1
done
cat gpurun_out/k_ab.jsonl
run 200 rocprofv3 --kernel-trace -d gpurun_out/st/k_c5 -o run --output-format csv \
  -- python tools/prof_step.py --config C5 --graphs 1 --steps 4 --graph > gpurun_out/k_st_c5.log 2>&1 || exit 1
python tools/step_timeline.py gpurun_out/st/k_c5/run_kernel_trace.csv > gpurun_out/st/k_c5.timeline.txt
cat gpurun_out/st/k_c5.timeline.txt
