#!/bin/bash
# Round-4 A/B session: 64-row head_bwd tiles (ab/hb64.so), head_fwd 64 vs 128 rows,
# window-SpMM neighbour chunk GK 2 / 4 / 8 (ab/gk2.so, default, ab/gk8.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
run 400 python -u -m pytest tests/test_gpu_step.py -k "fused_adam or replay" -x -q --timeout 300 > gpurun_out/fadam_tests.log 2>&1
echo "fused-adam tests rc=$?"; tail -3 gpurun_out/fadam_tests.log
run 300 python -u bench.py --steps 50 --warmup 5 > gpurun_out/bench_fadam.json 2> gpurun_out/bench_fadam.err
echo "bench rc=$?"; python -c "import json;j=json.loads(open('gpurun_out/bench_fadam.json').read().splitlines()[-1]);print(j['value'],j['ms_per_step'])"
SND_LIB_PATH=$PWD/ab/zpipe.so run 300 python -u -m pytest tests/test_gpu_ops.py -k "zzt" -x -q --timeout 200 > gpurun_out/zpipe_tests.log 2>&1
echo "zpipe tests rc=$?"; tail -2 gpurun_out/zpipe_tests.log
rm -f gpurun_out/ab.jsonl
run 400 bash tools/ab_multi.sh "--kernels zzt_dense --steps 100" 3 default ab/zpipe.so
python - <<PY
import json
for l in open("gpurun_out/ab.jsonl"):
    j = json.loads(l); print(j.get("tag", "?")[-14:], {k: v for k, v in j.items() if k != "tag"})
PY
SND_LIB_PATH=$PWD/ab/hb64.so run 400 python -u -m pytest tests/test_gpu_step.py -k "backward_head or c2_size or replay" -x -q --timeout 300 > gpurun_out/hb64_tests.log 2>&1
echo "hb64 tests rc=$?"; tail -2 gpurun_out/hb64_tests.log
rm -f gpurun_out/ab.jsonl
run 700 bash tools/ab_multi.sh "--kernels head_bwd,head_fwd --steps 100" 3 default ab/hb64.so
python - <<PY
import json
for l in open("gpurun_out/ab.jsonl"):
    j = json.loads(l); print(j.get("tag", "?")[-14:], {k: v for k, v in j.items() if k != "tag"})
PY
run 300 python tools/ab_fast.py --keys head_fwd,head_bwd --flags 0,131072,0,131072 2>&1 | grep -v amdgpu.ids
for r in 1; do
  for lib in ab/gk2.so default ab/gk8.so; do
    if [ "$lib" = default ]; then unset SND_LIB_PATH; else export SND_LIB_PATH=$PWD/$lib; fi
    echo "spmm $lib"; run 200 python tools/ab_spmm_win.py --flags 0 --rounds 3 2>&1 | grep "median"
  done
done
unset SND_LIB_PATH
echo done
