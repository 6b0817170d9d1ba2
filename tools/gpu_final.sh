#!/bin/bash
# Round-end evidence session: GPU tests, smoke, bench, rocprof (headline-only and full
# bench), PMC traffic, wgrad stamps (measurement library ab/meas.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGES="tests smoke bench profh traffic" bash tools/gpu_session.sh || exit $?
SND_LIB_PATH=$PWD/ab/meas.so timeout -k 10 200 python tools/wg_stamps.py --flags 0 > gpurun_out/wg_stamps.txt 2>gpurun_out/wg_stamps.err || exit $?
cat gpurun_out/wg_stamps.txt
