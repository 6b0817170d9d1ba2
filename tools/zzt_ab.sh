#!/bin/bash
# zz^T kernel trace: default build vs tools/_exp/$1.so, then the GPU zz^T tests on the variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/zab
KT="--kernel-trace --stats --output-format csv"
for v in base $1 base $1; do
  if [ $v = base ]; then unset SND_LIB_PATH; else export SND_LIB_PATH=$PWD/tools/_exp/$v.so; fi
  timeout -k 5 120 rocprofv3 $KT -d gpurun_out/zab/$v -o run -- python tools/prof_zzt.py \
    > gpurun_out/zab/$v.log 2>&1 || { echo "FAILED $v"; tail -20 gpurun_out/zab/$v.log; exit 1; }
  echo $v; grep -h "zzt_dense_bf16_v3" gpurun_out/zab/$v/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
done
export SND_LIB_PATH=$PWD/tools/_exp/$1.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_step.py \
  > gpurun_out/zab/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/zab/tests.log; exit 1; }
tail -1 gpurun_out/zab/tests.log
