# round 6: kernel trace of the frame calls on the mixed config's 2M frames in
# HBM (bench.py --frames without the crossover), and the diag line beside it
cd $GRAFT_REPO_ROOT || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_frames -o frames -- python3 bench.py --workload mixed --frames --no-crossover --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/frames_trace_line.json 2> gpurun_out/frames_trace.err
