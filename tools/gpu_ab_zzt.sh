#!/bin/bash
# zz^T A/B: ab/<lib>.so variants against the in-tree default (parity first, then timing
# in alternating processes).  usage: gpu_ab_zzt.sh lib1 [lib2 ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
libs=""
for v in "$@"; do
  SND_LIB_PATH=$PWD/ab/$v.so run 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py -k "zzt or c2_bench" -x -q --timeout 250 > gpurun_out/${v}_tests.log 2>&1
  echo "$v tests rc=$?"; tail -1 gpurun_out/${v}_tests.log
  libs="$libs ab/$v.so"
done
rm -f gpurun_out/ab.jsonl
run 600 bash tools/ab_multi.sh "--kernels zzt_dense --steps 200" ${ROUNDS:-3} default $libs
python - <<'PY'
import json, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/ab.jsonl"):
    j = json.loads(l)
    for k, v in j.items():
        if k.endswith("_us") or k.endswith("_ms"):
            d[j["tag"].split("/")[-1]][k].append(v)
for t, kv in d.items():
    print(t, {k: sorted(v) for k, v in kv.items()})
PY
echo done
