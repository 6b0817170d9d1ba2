#!/bin/bash
# Round 6, session A: GPU tests with the measured bars (recording every bf16 error),
# the broken-edge library against the C2 bench-batch test (must fail), the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/parity_errors.jsonl
STAGES="tests" bash tools/gpu_session.sh || exit $?
cp gpurun_out/parity_errors.jsonl gpurun_out/parity_errors_main.jsonl
echo "== broken-edge library (expected: FAIL)"
SND_LIB_PATH=$PWD/ab/edge_broken.so timeout -k 10 400 python -u -m pytest tests/test_gpu_c2_bench.py \
  -k bf16 -x -v --timeout 900 --timeout-method thread > gpurun_out/edge_broken_c2.log 2>&1
rc=$?
echo "== broken exit $rc"; tail -n 25 gpurun_out/edge_broken_c2.log | cut -c1-800
case $rc in 124|134|137|139) exit $rc;; esac
cp gpurun_out/parity_errors.jsonl gpurun_out/parity_errors_all.jsonl
STAGES="smoke bench" bash tools/gpu_session.sh
# A/B: the library built without SLP vectorisation (no v_pk_*_f32 in the epilogues)
# against HEAD, alternating processes, step + chain kernels
rm -f gpurun_out/ab.jsonl
bash tools/ab.sh "--kernels zzt_dense,head_fwd,head_bwd,dec:fwd,dec:bwd,wgrad_multi" ab/base.so ab/noslp.so 3
# A/B: the dec_fwd head phase on 4 threads per row
bash tools/ab.sh "--kernels dec:fwd" ab/base.so ab/decheads.so 3
bash tools/ab.sh "--kernels dec:fwd --graphs 1" ab/base.so ab/decheads.so 2
# zz^T symmetric-tile evidence: the v9 phase-skip proxy and the slab microbenchmark
timeout -k 10 300 python -u tools/ab_zzt.py --rounds 3 --reps 20 \
  --variants zzt_dense,zzt_dense_v256,zzt_dense_v1024,zzt_dense_v4096 > gpurun_out/zzt_sym_proxy.txt 2>&1
echo "== zzt proxy exit $?"; tail -12 gpurun_out/zzt_sym_proxy.txt
timeout -k 10 120 tools/micro/slab_cost > gpurun_out/slab_cost.json 2>&1; echo "== slab exit $?"; cat gpurun_out/slab_cost.json
# graph-replay kernel traces (the bench's own path, side streams as captured): B = 1 and 8
for B in 1 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/st/g$B -o run --output-format csv \
    -- python tools/prof_step.py --graphs $B --steps 6 --graph > gpurun_out/st_g$B.log 2>&1
  rc=$?; echo "== trace B=$B exit $rc"; case $rc in 124|134|137|139) exit $rc;; esac
  python tools/step_timeline.py gpurun_out/st/g$B/run_kernel_trace.csv > gpurun_out/st/g$B.timeline.txt && cat gpurun_out/st/g$B.timeline.txt
done
# one-graph step (C3 per rank): side stream at the highest priority or not, alternating
for r in 1 2 3; do
  for pr in 0 1; do
    SND_SIDE_PRIO=$pr timeout -k 10 180 python tools/ab_run.py --graphs 1 --kernels zzt_dense --tag prio$pr \
      >> gpurun_out/ab_prio.jsonl 2>> gpurun_out/ab_prio.err || { echo "prio run failed"; tail -5 gpurun_out/ab_prio.err; break 2; }
    tail -1 gpurun_out/ab_prio.jsonl | cut -c1-160
  done
done
SND_SIDE_PRIO=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/st/g1p -o run --output-format csv \
  -- python tools/prof_step.py --graphs 1 --steps 6 --graph > gpurun_out/st_g1p.log 2>&1 && \
  python tools/step_timeline.py gpurun_out/st/g1p/run_kernel_trace.csv > gpurun_out/st/g1p.timeline.txt && cat gpurun_out/st/g1p.timeline.txt
