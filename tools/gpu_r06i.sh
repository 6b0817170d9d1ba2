#!/bin/bash
# Round 6, session I: wgrad_multi with raised wave priority until the first unit lands
# (ab/prio.so, -DSND_WG_PRIO=1) against the shipped library; C2 step + the plan's
# wgrad_multi back to back, alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
for i in 1 2 3; do
  run 200 python tools/ab_run.py --kernels wgrad_multi --tag base >> gpurun_out/i_prio.jsonl 2>>gpurun_out/i_err.log || exit 1
  SND_LIB_PATH=ab/prio.so run 200 python tools/ab_run.py --kernels wgrad_multi --tag prio >> gpurun_out/i_prio.jsonl 2>>gpurun_out/i_err.log || exit 1
  SND_LIB_PATH=ab/spread.so run 200 python tools/ab_run.py --kernels wgrad_multi --tag spread >> gpurun_out/i_prio.jsonl 2>>gpurun_out/i_err.log || exit 1
done
cat gpurun_out/i_prio.jsonl
# enc_front at B = 7 (224 tiles + the pack workgroups fit 256 CUs one each) against B = 8
# (27 CUs run a tile and a pack workgroup together): graph-replay kernel traces
SND_LIB_PATH=ab/spread.so run 200 rocprofv3 --kernel-trace -d gpurun_out/st/i_g8s -o run --output-format csv \
  -- python tools/prof_step.py --graphs 8 --steps 6 --graph > gpurun_out/i_st_g8s.log 2>&1 || exit 1
python tools/step_timeline.py gpurun_out/st/i_g8s/run_kernel_trace.csv > gpurun_out/st/i_g8s.timeline.txt
head -3 gpurun_out/st/i_g8s.timeline.txt
for b in 7 8; do
  run 200 rocprofv3 --kernel-trace -d gpurun_out/st/i_g$b -o run --output-format csv \
    -- python tools/prof_step.py --graphs $b --steps 6 --graph > gpurun_out/i_st_g$b.log 2>&1 || exit 1
  python tools/step_timeline.py gpurun_out/st/i_g$b/run_kernel_trace.csv > gpurun_out/st/i_g$b.timeline.txt
  head -3 gpurun_out/st/i_g$b.timeline.txt
done
