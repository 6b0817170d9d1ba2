cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  timeout -k 10 180 python tools/ab_run.py --config C4 --kernels zzt_dense >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit 1
  timeout -k 10 180 python tools/ab_run.py --config C4 --kernels zzt_dense --adam-per-range >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit 1
done
echo done
