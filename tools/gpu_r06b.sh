#!/bin/bash
# Round 6, session B: the fp32 step-3 kink diagnostic, the one-graph concurrency swap A/B
# (+ replay trace), the dec_fwd head / partial-lane A/B, the edge-only broken library
# against the C2 bench-batch bf16 test (must fail), and the whole GPU suite (no -x: every
# bf16 case records its errors for tests/parity_bars.json).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
echo "== diag_kink"
run 400 python -u tools/diag_kink.py > gpurun_out/diag_kink.jsonl 2> gpurun_out/diag_kink.err
echo "rc=$?"; cut -c1-900 gpurun_out/diag_kink.jsonl; tail -3 gpurun_out/diag_kink.err
echo "== one-graph swap A/B"
rm -f gpurun_out/ab_swap.jsonl
for r in 1 2 3; do
  for dbg in 0 131072; do
    run 180 python tools/ab_run.py --graphs 1 --kernels dec:fwd --step-debug $dbg --tag b1 >> gpurun_out/ab_swap.jsonl 2>> gpurun_out/ab_swap.err
    tail -1 gpurun_out/ab_swap.jsonl | cut -c1-120
  done
done
run 200 rocprofv3 --kernel-trace -d gpurun_out/st/g1s -o run --output-format csv \
  -- python tools/prof_step.py --graphs 1 --steps 6 --graph --debug 131072 > gpurun_out/st_g1s.log 2>&1
python tools/step_timeline.py gpurun_out/st/g1s/run_kernel_trace.csv > gpurun_out/st/g1s.timeline.txt; cat gpurun_out/st/g1s.timeline.txt
echo "== dec heads A/B (base vs HEAD)"
rm -f gpurun_out/ab.jsonl
bash tools/ab.sh "--kernels dec:fwd" ab/base.so default 3
bash tools/ab.sh "--kernels dec:fwd --graphs 1" ab/base.so default 2
echo "== edge-only broken library (expected: FAIL on own_structure)"
SND_LIB_PATH=$PWD/ab/edge_broken.so run 400 python -u -m pytest tests/test_gpu_c2_bench.py \
  -k bf16 -x -v --timeout 900 --timeout-method thread > gpurun_out/edge_broken_c2.log 2>&1
echo "broken rc=$?"; grep -o "AssertionError: .*" gpurun_out/edge_broken_c2.log | cut -c1-700
echo "== pytest -m gpu (all cases)"
rm -f gpurun_out/parity_errors.jsonl
run 900 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -8 gpurun_out/pytest_gpu.log
