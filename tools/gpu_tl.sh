#!/bin/bash
# GPU tests of the reduce / step code, then step timelines: C2 at B = 8 and B = 4, C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/st
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
if [ -n "$TESTS" ]; then
  run 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/tl_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tl_tests.log; [ $rc = 0 ] || exit $rc
fi
for c in "c2b8:--graphs 8" "c2b4:--graphs 4" "c2b1:--graphs 1" "c5:--config C5 --graphs 1"; do
  n=${c%%:*}; a=${c#*:}
  [ -n "$ONLY" ] && [ "$ONLY" != "$n" ] && continue
  run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/st/$n -o run --output-format csv -- python tools/prof_step.py --steps 4 $a > gpurun_out/st/$n.log 2>&1 || exit $?
  python tools/step_timeline.py gpurun_out/st/$n/run_kernel_trace.csv > gpurun_out/st/$n.timeline.txt
  echo "== $n"; cat gpurun_out/st/$n.timeline.txt
done
