#!/bin/bash
# Round 6, session P: the reduction's loads in flight per round (SND_RED_RL, part lanes
# SND_RED_PL) against the shipped 8 / 2: C2 step, alternating processes, then the
# captured steps' kernel traces of the shipped and the best build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/st
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
for i in 1 2 3; do
  run 200 python tools/ab_run.py --kernels "" --tag base >> gpurun_out/p_ab.jsonl 2>>gpurun_out/p_err.log || exit 1
  for v in rl16 rl32 rl32_pl1 rl16_pl4; do
    SND_LIB_PATH=ab/$v.so run 200 python tools/ab_run.py --kernels "" --tag $v >> gpurun_out/p_ab.jsonl 2>>gpurun_out/p_err.log || exit 1
  done
done
grep -o '"tag": "[a-z0-9_]*", "step_ms": [0-9.]*' gpurun_out/p_ab.jsonl
for v in base rl16 rl32 rl32_pl1 rl16_pl4; do
  lib=ab/$v.so; [ $v = base ] && lib=snd_vae_amd/libsndvae.so
  SND_LIB_PATH=$PWD/$lib run 200 rocprofv3 --kernel-trace -d gpurun_out/st/p_$v -o run --output-format csv \
    -- python tools/prof_step.py --graphs 8 --steps 6 --graph > gpurun_out/p_st_$v.log 2>&1 || exit 1
  python tools/step_timeline.py gpurun_out/st/p_$v/run_kernel_trace.csv > gpurun_out/st/p_$v.timeline.txt
  echo "## $v"; tail -2 gpurun_out/st/p_$v.timeline.txt | cut -c1-110
done
