#!/bin/bash
# Round 6, session R: the step's weight images inside the gcn0 launch (C5, d = 128) --
# its parity test and the C5 tests, then the C5 step against pack_kernel before gcn0
# (host debug bit 1 << 28 at plan creation), alternating processes, and the C5 timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/st
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
run 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_configs.py \
  -k "gcn0 or c5 or 128" > gpurun_out/r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels "" --tag gcn0pack >> gpurun_out/r_ab.jsonl 2>>gpurun_out/r_err.log || exit 1
  run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels "" --step-debug 268435456 --tag packk >> gpurun_out/r_ab.jsonl 2>>gpurun_out/r_err.log || exit 1
done
# the reduction's part lanes for wide < 64-part slabs (C5's and the one-graph step's
# 32-chunk weight slabs): ab/plw2.so, ab/plw1.so against the shipped 4
for i in 1 2 3; do
  for v in base plw2 plw1; do
    lib=ab/$v.so; [ $v = base ] && lib=snd_vae_amd/libsndvae.so
    SND_LIB_PATH=$PWD/$lib run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels "" --tag c5_$v >> gpurun_out/r_ab.jsonl 2>>gpurun_out/r_err.log || exit 1
    SND_LIB_PATH=$PWD/$lib run 200 python tools/ab_run.py --graphs 1 --kernels "" --tag g1_$v >> gpurun_out/r_ab.jsonl 2>>gpurun_out/r_err.log || exit 1
  done
done
grep -o '"tag": "[a-z0-9_ ]*", "step_ms": [0-9.]*' gpurun_out/r_ab.jsonl
run 200 rocprofv3 --kernel-trace -d gpurun_out/st/r_c5 -o run --output-format csv \
  -- python tools/prof_step.py --config C5 --graphs 1 --steps 4 --graph > gpurun_out/r_st_c5.log 2>&1 || exit 1
python tools/step_timeline.py gpurun_out/st/r_c5/run_kernel_trace.csv > gpurun_out/st/r_c5.timeline.txt
cat gpurun_out/st/r_c5.timeline.txt
