#!/bin/bash
# Round-4 GPU session: GPU tests, bench (+ rocprof of the headline), one box.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139|-6|-11) return 0;; *) return 1;; esac; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"
  tail -n 4 "gpurun_out/$name.log"
  if fatal $rc; then echo "FATAL in $name ($rc), stopping"; exit $rc; fi
  return 0
}
STAGES=${STAGES:-"tests bench"}
for s in $STAGES; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) rm -f gpurun_out/parity_errors.jsonl
           step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    bench) step bench 600 python bench.py ;;
    benchq) step benchq 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --batch-sweep "" --extra "" ;;
    prof)  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run \
             --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra "" --batch-sweep "" --no-modes ;;
    abzzt) step ab_zzt 300 python tools/ab_zzt.py --variants ${ZZT_VARIANTS:-zzt_dense} --rounds 5 ;;
    abspmm) step ab_spmm 300 python tools/ab_spmm_win.py --flags ${SPMM_FLAGS:-0} --rounds 6 ;;
    some) step pytest_some 600 python -u -m pytest ${TESTS} -x -v --timeout 300 --timeout-method thread ;;
    abfast) step ab_fast 300 python tools/ab_fast.py --keys ${FAST_KEYS:-head_fwd,head_bwd} --flags ${FAST_FLAGS:-0} ;;
    strong) step strong 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --batch-sweep "" --extra "" ;;
  esac
done
echo "== done"
