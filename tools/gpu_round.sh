#!/bin/bash
# Round check on one MI355X: GPU tests, smoke, the torchrun (RCCL) path with one
# rank and the all-reduce forced on, then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest_gpu"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
echo "== smoke"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "== torchrun world 1, forced all-reduce"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --force-dist --extra "" --no-cpu-baseline \
  > gpurun_out/bench_dist1.log 2>&1 || { echo "DIST BENCH FAILED"; tail -30 gpurun_out/bench_dist1.log; exit 1; }
tail -1 gpurun_out/bench_dist1.log | cut -c1-300
if [ -n "$BENCH" ]; then
  echo "== bench"
  timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log | cut -c1-400
fi
echo "== done"
