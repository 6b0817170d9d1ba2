#!/bin/bash
# Step-time A/B of plan-creation debug bits (tools/step_time.py --debug), alternating
# processes on one box.  usage: gpu_ab_dbg.sh "0 128" [extra step_time args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
rm -f gpurun_out/ab_dbg.jsonl
for r in $(seq ${ROUNDS:-3}); do
  for d in $1; do
    run 120 python -u tools/step_time.py --steps 300 --debug $d --tag dbg$d $2 >> gpurun_out/ab_dbg.jsonl 2>>gpurun_out/ab.err
  done
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab_dbg.jsonl"):
    j = json.loads(l); d[j["tag"]].append(j["ms_median"])
for k, v in d.items(): print(k, sorted(v))
PY
