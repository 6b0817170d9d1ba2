#!/bin/bash
# Round 6, session T: rowconv RC_ENC1 with one 16-byte load per whole P1 quad (C5's
# backward) against the previous tree (ab/prev.so): the C5 / d = 128 tests, the C5 step
# in alternating processes, the C5 timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/st
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
run 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_configs.py \
  tests/test_gpu_ops.py -k "c5 or 128 or rowconv or row_engine" > gpurun_out/t_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/t_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels "" --tag c5_new >> gpurun_out/t_ab.jsonl 2>>gpurun_out/t_err.log || exit 1
  SND_LIB_PATH=$PWD/ab/prev.so run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels "" --tag c5_prev >> gpurun_out/t_ab.jsonl 2>>gpurun_out/t_err.log || exit 1
done
grep -o '"tag": "[a-z0-9_ ]*", "step_ms": [0-9.]*' gpurun_out/t_ab.jsonl
for v in new prev; do
  lib=ab/prev.so; [ $v = new ] && lib=snd_vae_amd/libsndvae.so
  SND_LIB_PATH=$PWD/$lib run 200 rocprofv3 --kernel-trace -d gpurun_out/st/t_$v -o run --output-format csv \
    -- python tools/prof_step.py --config C5 --graphs 1 --steps 4 --graph > gpurun_out/t_st_$v.log 2>&1 || exit 1
  python tools/step_timeline.py gpurun_out/st/t_$v/run_kernel_trace.csv > gpurun_out/st/t_$v.timeline.txt
  echo "## $v"; grep "rowconv_kernel<3" gpurun_out/st/t_$v.timeline.txt; tail -1 gpurun_out/st/t_$v.timeline.txt
done
