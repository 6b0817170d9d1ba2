#!/bin/bash
# Step-time A/B over the C2, one-graph (C3 per rank) and C5 workloads: in-tree vs $LIB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
if [ -n "$TESTS" ]; then
  run 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/cfgab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/cfgab_tests.log; [ $rc = 0 ] || exit $rc
fi
rm -f gpurun_out/cfgab.jsonl
for r in 1 2; do
  for lib in default $LIB; do
    if [ "$lib" = default ]; then unset SND_LIB_PATH; else export SND_LIB_PATH=$PWD/$lib; fi
    run 200 python tools/ab_run.py --config C5 --graphs 1 --kernels "" --tag C5:$lib >> gpurun_out/cfgab.jsonl 2>>gpurun_out/cfgab.err
    run 200 python tools/ab_run.py --graphs 1 --kernels "" --tag B1:$lib >> gpurun_out/cfgab.jsonl 2>>gpurun_out/cfgab.err
    run 200 python tools/ab_run.py --kernels "" --tag C2:$lib >> gpurun_out/cfgab.jsonl 2>>gpurun_out/cfgab.err
  done
done
unset SND_LIB_PATH
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/cfgab.jsonl"):
    j = json.loads(l); d[j["tag"]].append(j["step_ms"])
for k, v in sorted(d.items()): print(k, sorted(v))
PY
