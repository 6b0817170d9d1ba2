cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/st
for c in C2 C4 C5; do
  a=""; [ $c != C2 ] && a="--config $c"; [ $c == C5 ] && a="$a --graphs 1"
  timeout -k 5 120 rocprofv3 --kernel-trace --stats -d gpurun_out/st/$c -o run --output-format csv -- python tools/prof_step.py --steps 4 $a > gpurun_out/st/$c.log 2>&1 || { echo FAIL $c; exit 1; }
  python tools/step_timeline.py gpurun_out/st/$c/run_kernel_trace.csv > gpurun_out/st/$c.timeline.txt
done
echo done
