# C4 step timeline + the graph-latent / fused-Adam GPU tests
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/st4
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_dp.py tests/test_gpu_sgjoint.py > gpurun_out/t4.log 2>&1 || { echo TESTS FAILED; exit 1; }
timeout -k 5 150 rocprofv3 --kernel-trace --stats -d gpurun_out/st4/C4 -o run --output-format csv -- python tools/prof_step.py --steps 4 --config C4 > gpurun_out/st4/C4.log 2>&1 && python tools/step_timeline.py gpurun_out/st4/C4/run_kernel_trace.csv > gpurun_out/st4/C4.timeline.txt && echo done
