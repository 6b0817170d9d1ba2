#!/bin/bash
# Round 6, session F: the fused decoder beside zz^T at C2 (B = 8, plan option conc_decoder=1)
# with the 128-row decoder (one 148 KB workgroup per CU: it cannot share a CU with zz^T) and
# with the reverted dual decoder (ab/dual.so, snd_dec.* of commit 56f1efd on the current tree: 76 KB, 8 waves -- one zz^T and
# one decoder workgroup fit a CU together); alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if fatal $rc; then echo "FATAL $rc: $*"; exit $rc; fi; return $rc; }
for i in 1 2 3; do
  run 200 python tools/ab_run.py --kernels zzt_dense --tag serial >> gpurun_out/f_conc.jsonl 2>>gpurun_out/f_err.log || exit 1
  run 200 python tools/ab_run.py --kernels zzt_dense --tag conc --option conc_decoder=1 >> gpurun_out/f_conc.jsonl 2>>gpurun_out/f_err.log || exit 1
  SND_LIB_PATH=ab/dual.so run 200 python tools/ab_run.py --kernels zzt_dense --tag dual-conc --option conc_decoder=1 >> gpurun_out/f_conc.jsonl 2>>gpurun_out/f_err.log || exit 1
done
cat gpurun_out/f_conc.jsonl
