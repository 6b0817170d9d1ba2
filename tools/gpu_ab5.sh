#!/bin/bash
# Round-5 A/B session over the round-4 variants, rebuilt from HEAD (tools/build_ab.sh):
# zzT v4 software-pipelined tile (ab/zpipe.so), 64-row backward-head tiles (ab/hb64.so),
# window-SpMM neighbour chunk 2 / 4 / 8 (ab/gk2.so, default, ab/gk8.so), and the
# reduction-fused Adam on / off (plan option).  Alternating processes on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
summ() { python - "$1" <<'PY'
import json, sys, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open(sys.argv[1]):
    j = json.loads(l)
    for k, v in j.items():
        if k.endswith("_us") or k.endswith("_ms") or k == "ms_median":
            d[j["tag"].split("/")[-1]][k].append(v)
for t, kv in d.items():
    print(t, {k: sorted(v) for k, v in kv.items()})
PY
}
SND_LIB_PATH=$PWD/ab/zpipe.so run 300 python -u -m pytest tests/test_gpu_ops.py -k "zzt" -x -q --timeout 200 > gpurun_out/zpipe_tests.log 2>&1
echo "zpipe tests rc=$?"; tail -2 gpurun_out/zpipe_tests.log
for v in v9 v9s; do
  SND_LIB_PATH=$PWD/ab/$v.so run 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py -k "zzt or c2_bench" -x -q --timeout 250 > gpurun_out/${v}_tests.log 2>&1
  echo "$v tests rc=$?"; tail -2 gpurun_out/${v}_tests.log
done
SND_LIB_PATH=$PWD/ab/hb64.so run 400 python -u -m pytest tests/test_gpu_step.py -k "backward_head or c2_size or replay" -x -q --timeout 300 > gpurun_out/hb64_tests.log 2>&1
echo "hb64 tests rc=$?"; tail -2 gpurun_out/hb64_tests.log
rm -f gpurun_out/ab.jsonl
run 700 bash tools/ab_multi.sh "--kernels zzt_dense,head_bwd,head_fwd --steps 200" 3 default ab/zpipe.so ab/hb64.so ab/v9.so ab/v9s.so
summ gpurun_out/ab.jsonl
for r in 1 2; do
  for lib in ab/gk2.so default ab/gk8.so; do
    if [ "$lib" = default ]; then unset SND_LIB_PATH; else export SND_LIB_PATH=$PWD/$lib; fi
    echo "spmm $lib"; run 200 python tools/ab_spmm_win.py --flags 0 --rounds 3 2>&1 | grep "median"
  done
done
unset SND_LIB_PATH
rm -f gpurun_out/ab_radam.jsonl
for r in 1 2 3; do
  for o in 1 0; do
    run 120 python -u tools/step_time.py --steps 300 --option reduce_adam=$o --tag radam$o >> gpurun_out/ab_radam.jsonl 2>>gpurun_out/ab.err
  done
done
summ gpurun_out/ab_radam.jsonl
echo done
