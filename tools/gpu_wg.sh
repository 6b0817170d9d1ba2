#!/bin/bash
# wgrad split session: per-kernel A/B of wgrad_multi against ab/base.so (HEAD before
# the change) and step time at 64 / 32 row chunks (debug bit 16384), alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
rm -f gpurun_out/ab.jsonl gpurun_out/ab_step.jsonl
run 400 bash tools/ab_multi.sh "--kernels wgrad_multi --steps 100" 3 default ab/base.so
python - <<'PY'
import json, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/ab.jsonl"):
    j = json.loads(l)
    for k, v in j.items():
        if k.endswith("_us"): d[j["tag"]][k].append(v)
for t, kv in d.items(): print(t, {k: sorted(v) for k, v in kv.items()})
PY
for r in 1 2 3; do
  for d in 0 16384; do
    run 120 python -u tools/step_time.py --steps 300 --debug $d --tag chunks$d >> gpurun_out/ab_step.jsonl 2>>gpurun_out/ab.err
  done
  SND_LIB_PATH=$PWD/ab/base.so run 120 python -u tools/step_time.py --steps 300 --debug 16384 --tag base16384 >> gpurun_out/ab_step.jsonl 2>>gpurun_out/ab.err
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab_step.jsonl"):
    j = json.loads(l); d[j["tag"]].append(j["ms_median"])
for k, v in d.items(): print(k, sorted(v))
PY
