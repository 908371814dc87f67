#!/usr/bin/env bash
# Headline evidence for one round (GPU box): the default bench line, the
# rocprofv3 --kernel-trace --stats summary of the same command, and the PMC
# passes of the dominant kernel, for one workload.
#   TAG=r02 WL=tcp1500 KRE=k_window bash scripts/evidence.sh
# Outputs under gpurun_out/evidence_<tag>_<wl>/; every GPU step has its own
# time limit and the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
WL=${WL:-tcp1500}
KRE=${KRE:-k_window}
EXTRA=${EXTRA:-}
D=gpurun_out/evidence_${TAG}_${WL}
mkdir -p $D
step() { local rc; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
# 1. the bench line itself (default steps/warm-up, cpu_baseline included)
step timeout -k 10 180 python3 bench.py --workload $WL $EXTRA > $D/bench.json 2> $D/bench.err
# 2. the same command under the kernel trace
step timeout -k 10 240 /opt/rocm/bin/rocprofv3 --kernel-trace --stats -T --output-format csv \
    -d $D/trace -o trace -- python3 bench.py --workload $WL $EXTRA > $D/trace.json 2> $D/trace.err
# 3. PMC passes (one counter group per run), short runs
OUT=$D/prof KRE=$KRE BENCH="bench.py --workload $WL --steps 20 --warmup 3 --settle-ms 0 --no-cpu-baseline $EXTRA" \
    step bash scripts/profile.sh
echo "evidence in $D"
