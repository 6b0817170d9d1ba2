#!/bin/bash
# Round 6, session O: weight-gradient row chunks per kernel width.  wgrad_multi's
# per-workgroup stamps on the shipped geometry (ab/meas.so), then the C2 step + the
# plan's wgrad_multi for chunk-count builds (SND_WGC_T1 / SND_WGC_T5) against the
# shipped 64 / 64, alternating processes, and the captured steps' kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/st
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
SND_LIB_PATH=ab/meas.so run 200 python tools/wg_stamps.py > gpurun_out/o_stamps.txt 2>gpurun_out/o_stamps.err || exit 1
head -40 gpurun_out/o_stamps.txt
for i in 1 2 3; do
  run 200 python tools/ab_run.py --kernels wgrad_multi --tag base >> gpurun_out/o_ab.jsonl 2>>gpurun_out/o_err.log || exit 1
  for v in t1_32 t1_32_t5_96 t1_48 t5_96; do
    SND_LIB_PATH=ab/$v.so run 200 python tools/ab_run.py --kernels wgrad_multi --tag $v >> gpurun_out/o_ab.jsonl 2>>gpurun_out/o_err.log || exit 1
  done
done
cut -c1-60 gpurun_out/o_ab.jsonl; grep -o '"tag": "[a-z0-9_]*"\|"wgrad_multi_us": [0-9.]*' gpurun_out/o_ab.jsonl | paste - - 
for v in base t1_32 t1_32_t5_96; do
  lib=ab/$v.so; [ $v = base ] && lib=snd_vae_amd/libsndvae.so
  SND_LIB_PATH=$PWD/$lib run 200 rocprofv3 --kernel-trace -d gpurun_out/st/o_$v -o run --output-format csv \
    -- python tools/prof_step.py --graphs 8 --steps 6 --graph > gpurun_out/o_st_$v.log 2>&1 || exit 1
  python tools/step_timeline.py gpurun_out/st/o_$v/run_kernel_trace.csv > gpurun_out/st/o_$v.timeline.txt
  tail -4 gpurun_out/st/o_$v.timeline.txt
done
