#!/bin/bash
# Round 6, session N: zz^T v10 (d = 128: two 512-thread workgroups per CU) -- the zz^T,
# C5 and row-sharded tests, then the C5 step and the zz^T launch against v7
# (ab/v7.so, -DSND_ZZT_V10=0), alternating processes.  v10 lost and was reverted
# (profiles/r06_ab_zzt_v10_c5.txt); the script needs commit 7e251ff's tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
run 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_configs.py \
  tests/test_gpu_row_shard.py tests/test_gpu_row_shard_step.py -k "zzt or c5 or 128 or row" > gpurun_out/n_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/n_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels zzt_dense --tag v10 >> gpurun_out/n_ab.jsonl 2>>gpurun_out/n_err.log || exit 1
  SND_LIB_PATH=ab/v7.so run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels zzt_dense --tag v7 >> gpurun_out/n_ab.jsonl 2>>gpurun_out/n_err.log || exit 1
done
cat gpurun_out/n_ab.jsonl
run 200 rocprofv3 --kernel-trace -d gpurun_out/st/n_c5 -o run --output-format csv \
  -- python tools/prof_step.py --config C5 --graphs 1 --steps 4 --graph > gpurun_out/n_st_c5.log 2>&1 || exit 1
python tools/step_timeline.py gpurun_out/st/n_c5/run_kernel_trace.csv > gpurun_out/st/n_c5.timeline.txt
cat gpurun_out/st/n_c5.timeline.txt
