#!/bin/bash
# wgrad_multi phase skips (measurement builds): new split vs the previous tree, 64 / 32 chunks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/wg_meas.jsonl
for lib in meas meas_base; do
  SND_LIB_PATH=$PWD/ab/$lib.so timeout -k 10 200 python tools/ab_run.py --kernels wgrad_multi --debug 0,2,4,14,16384,16398 --tag $lib >> gpurun_out/wg_meas.jsonl 2>>gpurun_out/wg_meas.err || exit $?
done
cat gpurun_out/wg_meas.jsonl
