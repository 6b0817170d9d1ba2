#!/bin/bash
# Step-time A/B over (library, plan debug bits) variants, alternating processes:
#   VARIANTS="default:0 default:16384 ab/pl16.so:0" bash tools/gpu_abv.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
rm -f gpurun_out/abv.jsonl
for r in $(seq ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    lib=${v%%:*}; d=${v##*:}
    if [ "$lib" = default ]; then unset SND_LIB_PATH; else export SND_LIB_PATH=$PWD/$lib; fi
    run 120 python -u tools/step_time.py --steps 300 --debug $d --tag $v $STEPARGS >> gpurun_out/abv.jsonl 2>>gpurun_out/abv.err
  done
done
unset SND_LIB_PATH
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/abv.jsonl"):
    j = json.loads(l); d[j["tag"]].append(j["ms_median"])
for k, v in d.items(): print(k, sorted(v))
PY
