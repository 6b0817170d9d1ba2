#!/bin/bash
# One-graph (C3 per rank) step A/B: in-tree vs each library of $LIBS, alternating processes;
# $TESTS run first against the LAST library of $LIBS (SND_LIB_PATH).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
if [ -n "$TESTS" ]; then
  for l in $LIBS; do last=$l; done
  SND_LIB_PATH=$PWD/$last run 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/b1ab_tests.log 2>&1
  rc=$?; echo "tests ($last) rc=$rc"; tail -2 gpurun_out/b1ab_tests.log; [ $rc = 0 ] || exit $rc
fi
rm -f gpurun_out/b1ab.jsonl
for r in 1 2 3; do
  for lib in default $LIBS; do
    if [ "$lib" = default ]; then unset SND_LIB_PATH; else export SND_LIB_PATH=$PWD/$lib; fi
    run 200 python tools/ab_run.py --graphs ${GRAPHS:-1} --kernels "" --tag B${GRAPHS:-1}:$lib >> gpurun_out/b1ab.jsonl 2>>gpurun_out/b1ab.err
  done
done
unset SND_LIB_PATH
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/b1ab.jsonl"):
    j = json.loads(l); d[j["tag"]].append(j["step_ms"])
for k, v in sorted(d.items()): print(k, sorted(v))
PY
