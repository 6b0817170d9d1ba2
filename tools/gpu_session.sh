#!/bin/bash
# One GPU-box session, stage list in $STAGES (default: tests smoke ab bench timeline).
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
  tail -n ${TAILN:-6} "gpurun_out/$name.log" | cut -c1-600
  if fatal $rc; then echo "FATAL in $name ($rc), stopping"; exit $rc; fi
  [ $rc -ne 0 ] && [ -n "$STRICT" ] && exit $rc
  return 0
}

for s in ${STAGES:-tests smoke ab bench timeline}; do
  case $s in
    tests) step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    smoke) step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    ab) step ab 400 python -u tools/ab_flags.py --flags ${ABFLAGS:-0,32768} --kernels ${ABKERN:-zzt_dense} ;;
    bench) step bench 400 python -u bench.py ;;
    dist1) step bench_dist1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
             --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 \
             --force-dist --extra "" --no-cpu-baseline ;;
    timeline)
      for c in ${TLCONF:-C2}; do
        a=""; [ $c != C2 ] && a="--config $c"; [ $c == C5 ] && a="$a --graphs 1"
        step tl_$c 200 rocprofv3 --kernel-trace --stats -d gpurun_out/st/$c -o run --output-format csv \
          -- python tools/prof_step.py --steps 4 $a
        python tools/step_timeline.py gpurun_out/st/$c/run_kernel_trace.csv > gpurun_out/st/$c.timeline.txt
        tail -3 gpurun_out/st/$c.timeline.txt
      done ;;
    prof) step rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run \
             --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra "" ;;
    profh) step rocprof_headline 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profh -o run \
             --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra "" \
             --batch-sweep "" --no-modes ;;
    benchq) step benchq 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --batch-sweep "" --extra "" ;;
    traffic)   # per-kernel HBM bytes of eager C2 steps: one counter per rocprofv3 run
      step pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv \
        -- python tools/prof_step.py --steps 3
      step pmc_write 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv \
        -- python tools/prof_step.py --steps 3
      python tools/pmc_kernels.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/traffic_c2.json \
        --alg zzt_dense=17039360 --zzt-json gpurun_out/pmc_zzt_c2.json ;;
    sq) step pmc_sq 900 bash tools/pmc_step.sh ;;
    custom) step custom ${CUSTOM_SECS:-300} bash -c "$CUSTOM" ;;
  esac
done
echo "== done"
