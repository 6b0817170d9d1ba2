#!/bin/bash
# Round 6, session E: the window SpMM's deep-prefetch ring (1024 rows, slot lists two
# steps ahead) -- bitwise tests of both rings, the kernel A/B on the 256-graph batch and
# its phase skips -- and the dual decoder tiles (64 rows, 8 waves, weights streamed by
# tap, two workgroups per CU): the fused-decoder tests and a C2 step A/B in alternating
# processes against the 16-wave 64-row kernels (host bit 1 << 18) and the 128-row tiles
# (ab/nodual.so, -DSND_DEC_DUAL=0); 64-row backward-head tiles (ab/hb64.so, -DSND_HB_SMALL=100000,
# built from the dual-decoder sources).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
run 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_step.py -k "window or fused_decoder" \
  > gpurun_out/e_step.log 2>&1
rc=$?; echo "step rc=$rc"; tail -4 gpurun_out/e_step.log; [ $rc -ne 0 ] && exit $rc
run 300 python -u tools/ab_spmm_win.py --rings 1096,1024 --flags 0 --rounds 5 > gpurun_out/e_rings.txt 2>&1
echo "rings rc=$?"; tail -4 gpurun_out/e_rings.txt
run 300 python -u tools/ab_spmm_win.py --rings 1024 --flags 0,16777216,33554432,67108864,100663296 --rounds 3 \
  > gpurun_out/e_deep_skips.txt 2>&1
echo "skips rc=$?"; tail -6 gpurun_out/e_deep_skips.txt
for i in 1 2 3; do
  run 200 python tools/ab_run.py --kernels dec:fwd,dec:bwd --tag dual >> gpurun_out/e_dec_ab.jsonl 2>>gpurun_out/e_dec_err.log || exit 1
  run 200 python tools/ab_run.py --kernels dec:fwd,dec:bwd --tag w16t64 --step-debug 262144 >> gpurun_out/e_dec_ab.jsonl 2>>gpurun_out/e_dec_err.log || exit 1
  SND_LIB_PATH=ab/nodual.so run 200 python tools/ab_run.py --kernels dec:fwd,dec:bwd --tag t128 >> gpurun_out/e_dec_ab.jsonl 2>>gpurun_out/e_dec_err.log || exit 1
  SND_LIB_PATH=ab/hb64.so run 200 python tools/ab_run.py --kernels dec:fwd,dec:bwd,head_bwd --tag hb64 >> gpurun_out/e_dec_ab.jsonl 2>>gpurun_out/e_dec_err.log || exit 1
done
cat gpurun_out/e_dec_ab.jsonl
