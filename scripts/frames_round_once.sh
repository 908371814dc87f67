# After a frame-call change: the -m gpu suite, smoke() and the default bench
# line (scripts/gpu_round.sh), the frame-shape A/B, then the --frames profile
# (trace + PMC passes) for scripts/frames_summary.py.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit $?
timeout -k 10 300 python scripts/lab_frames_ab.py gpurun_out/frames_ab2.json 7 > gpurun_out/frames_ab2.log 2>&1
rc=$?; grep -E " us " gpurun_out/frames_ab2.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/frames_ab2.log; exit $rc; }
OUT=gpurun_out/prof_frames KRE="k_flat2|k_rx_hdr" BENCH="bench.py --frames --steps 5 --warmup 2 --no-cpu-baseline" bash scripts/profile.sh
