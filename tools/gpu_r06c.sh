#!/bin/bash
# Round 6, session C: the whole GPU suite on HEAD (measured bars, fp32 kink ties), the
# dec_fwd head A/B (base = before the change), smoke and the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
rm -f gpurun_out/parity_errors.jsonl gpurun_out/ab.jsonl
echo "== pytest -m gpu"
run 900 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gpu.log; grep -o "AssertionError: .*" gpurun_out/pytest_gpu.log | cut -c1-600
echo "== dec heads A/B"
bash tools/ab.sh "--kernels dec:fwd" ab/base.so default 3
bash tools/ab.sh "--kernels dec:fwd --graphs 1" ab/base.so default 3
STAGES="smoke bench" bash tools/gpu_session.sh
