cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dp/pytest.log 2>&1 || { tail -30 gpurun_out/dp/pytest.log; exit 1; }
tail -3 gpurun_out/dp/pytest.log
for v in "--buckets" ""; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --force-dist --extra C4 --no-modes --batch-sweep "" --no-cpu-baseline $v > gpurun_out/dp/dist$v.log 2>&1 || { tail -30 gpurun_out/dp/dist$v.log; exit 1; }
  grep "\[C4\]" gpurun_out/dp/dist$v.log | cut -c1-200
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra C4 --no-modes --batch-sweep "" --no-cpu-baseline > gpurun_out/dp/single.log 2>&1 || { tail -30 gpurun_out/dp/single.log; exit 1; }
grep "\[C4\]" gpurun_out/dp/single.log | cut -c1-200
