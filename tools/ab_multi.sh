#!/bin/bash
# Alternating A/B over several libraries: ab_multi.sh "ARGS" rounds lib1 lib2 ... ('default' = in-tree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
args=$1; rounds=$2; shift 2
for r in $(seq $rounds); do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset SND_LIB_PATH; else export SND_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 180 python tools/ab_run.py $args >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || { echo "FAILED $lib"; tail -20 gpurun_out/ab.err; exit 1; }
  done
done
echo done
