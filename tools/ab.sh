#!/bin/bash
# Alternating A/B processes on the GPU box: ab.sh "ARGS" libA libB [rounds]
# (each lib path or 'default'); one JSON line per process into gpurun_out/ab.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
args=$1; a=$2; b=$3; rounds=${4:-3}
for r in $(seq $rounds); do
  for lib in $a $b; do
    if [ "$lib" = default ]; then unset SND_LIB_PATH; else export SND_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 180 python tools/ab_run.py $args >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || { echo "FAILED $lib"; tail -20 gpurun_out/ab.err; exit 1; }
    tail -1 gpurun_out/ab.jsonl | cut -c1-200
  done
done
