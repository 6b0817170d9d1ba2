#!/bin/bash
# parity tests on the in-tree library, then step time: in-tree vs ab/prev.so vs ab/base.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
if [ -n "$TESTS" ]; then
  run 500 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/ab3_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ab3_tests.log; [ $rc = 0 ] || exit $rc
fi
rm -f gpurun_out/ab_step.jsonl
for r in 1 2 3; do
  for lib in default ${LIBS:-ab/prev.so ab/base.so}; do
    if [ "$lib" = default ]; then unset SND_LIB_PATH; else export SND_LIB_PATH=$PWD/$lib; fi
    run 120 python -u tools/step_time.py --steps 300 --tag $lib $STEPARGS >> gpurun_out/ab_step.jsonl 2>>gpurun_out/ab.err
  done
done
unset SND_LIB_PATH
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab_step.jsonl"):
    j = json.loads(l); d[j["tag"]].append(j["ms_median"])
for k, v in d.items(): print(k, sorted(v))
PY
if [ -n "$KERNELS" ]; then
  rm -f gpurun_out/ab.jsonl
  run 400 bash tools/ab_multi.sh "--kernels $KERNELS --steps 100" 2 default ${LIBS:-ab/prev.so ab/base.so}
  python - <<'PY'
import json, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/ab.jsonl"):
    j = json.loads(l)
    for k, v in j.items():
        if k.endswith("_us"): d[j["tag"]][k].append(v)
for t, kv in d.items(): print(t, {k: sorted(v) for k, v in kv.items()})
PY
fi
