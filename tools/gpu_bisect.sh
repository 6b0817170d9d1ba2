#!/bin/bash
# Round-5 regression bisect: C2 B=8 step time of several source trees (each with its own
# prebuilt libsndvae.so under _bisect/<sha>/), alternating processes on one box, then an
# eager kernel trace of the oldest and newest tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
TREES=${TREES:-"_bisect/7654dd2 _bisect/cd0a5a5 _bisect/29e077a _bisect/88ca195 _bisect/7fe8025 _bisect/f857f28 _bisect/c0c80db ."}
ROUNDS=${ROUNDS:-3}
rm -f gpurun_out/bisect.jsonl
for r in $(seq $ROUNDS); do
  for t in $TREES; do
    run 120 python -u tools/step_time.py --root $t --steps 300 --tag "$t" >> gpurun_out/bisect.jsonl 2>> gpurun_out/bisect.err
  done
  echo "round $r done"
done
python - <<PY
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/bisect.jsonl"):
    j = json.loads(l); d[j["tag"]].append(j["ms_median"])
for k, v in d.items():
    print(f"{k:24s} {sorted(v)}")
PY
for t in ${PROF_TREES:-_bisect/7654dd2 .}; do
  name=$(basename $t); [ "$name" = . ] && name=head
  run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- python tools/step_time.py --root $t --eager 5 > gpurun_out/prof_$name.log 2>&1
  echo "prof $name rc=$?"
done
echo done
