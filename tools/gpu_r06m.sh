#!/bin/bash
# Round 6, session M: reparam_prep on 1024-thread blocks (C5) -- the encoder-head and C5 tests,
# then the C5 step against the 256-thread kernel (ab/prep256.so), alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
run 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_configs.py \
  -k "encoder_head or c5 or 128 or edge_terms" > gpurun_out/m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/m_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels zzt_dense --tag prep1024 >> gpurun_out/m_ab.jsonl 2>>gpurun_out/m_err.log || exit 1
  SND_LIB_PATH=ab/prep256.so run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels zzt_dense --tag prep256 >> gpurun_out/m_ab.jsonl 2>>gpurun_out/m_err.log || exit 1
done
cat gpurun_out/m_ab.jsonl
run 200 rocprofv3 --kernel-trace -d gpurun_out/st/m_c5 -o run --output-format csv \
  -- python tools/prof_step.py --config C5 --graphs 1 --steps 4 --graph > gpurun_out/m_st_c5.log 2>&1 || exit 1
python tools/step_timeline.py gpurun_out/st/m_c5/run_kernel_trace.csv > gpurun_out/st/m_c5.timeline.txt
cat gpurun_out/st/m_c5.timeline.txt
