#!/bin/bash
# Round 6, session Q: enc_front with its tiles' waves at a raised priority (s_setprio 1 / 3,
# ab/fprio*.so) against the shipped library, whose 27 pack workgroups share CUs with
# tiles at C2: C2 step in alternating processes, then captured-step kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/st
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
for i in 1 2 3; do
  run 200 python tools/ab_run.py --kernels "" --tag base >> gpurun_out/q_ab.jsonl 2>>gpurun_out/q_err.log || exit 1
  for v in fprio1 fprio3; do
    SND_LIB_PATH=ab/$v.so run 200 python tools/ab_run.py --kernels "" --tag $v >> gpurun_out/q_ab.jsonl 2>>gpurun_out/q_err.log || exit 1
  done
done
grep -o '"tag": "[a-z0-9_]*", "step_ms": [0-9.]*' gpurun_out/q_ab.jsonl
for v in base fprio1 fprio3; do
  lib=ab/$v.so; [ $v = base ] && lib=snd_vae_amd/libsndvae.so
  SND_LIB_PATH=$PWD/$lib run 200 rocprofv3 --kernel-trace -d gpurun_out/st/q_$v -o run --output-format csv \
    -- python tools/prof_step.py --graphs 8 --steps 6 --graph > gpurun_out/q_st_$v.log 2>&1 || exit 1
  python tools/step_timeline.py gpurun_out/st/q_$v/run_kernel_trace.csv > gpurun_out/st/q_$v.timeline.txt
  echo "## $v"; head -2 gpurun_out/st/q_$v.timeline.txt | cut -c1-110; tail -1 gpurun_out/st/q_$v.timeline.txt
done
