cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/st5b
timeout -k 5 150 rocprofv3 --kernel-trace --stats -d gpurun_out/st5b/C5 -o run --output-format csv -- python tools/prof_step.py --steps 4 --config C5 --graphs 1 > gpurun_out/st5b/C5.log 2>&1 && python tools/step_timeline.py gpurun_out/st5b/C5/run_kernel_trace.csv > gpurun_out/st5b/C5.timeline.txt && echo done
