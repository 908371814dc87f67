#!/usr/bin/env bash
# rocprofv3 evidence for the bench's checksum kernel (run on the GPU box):
#   1. kernel trace + stats of the bench command itself  -> gpurun_out/prof/trace
#   2. SQ instruction / wait counters (own pass)          -> gpurun_out/prof/sq
#   3. FETCH_SIZE (own pass; gfx950 reports 1/2 of wide streaming reads)
#   4. WRITE_SIZE (own pass)
#   (optional) SQ2="..." a second SQ counter pass, before 3
# Each pass runs under its own time limit; anything but success/plain failure
# (rc 0/1) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
BENCH=${BENCH:-"bench.py --steps 20 --warmup 3 --no-cpu-baseline"}
KRE=${KRE:-k_stream}
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 ${PROF_TIMEOUT:-240} /opt/rocm/bin/rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 $BENCH > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"; tail -2 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run trace --kernel-trace --stats -T
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$KRE" -T
if [ -n "${SQ2:-}" ]; then run sq2 --pmc $SQ2 --kernel-include-regex "$KRE" -T; fi
run fetch --pmc FETCH_SIZE --kernel-include-regex "$KRE" -T
run write --pmc WRITE_SIZE --kernel-include-regex "$KRE" -T
find $OUT -name "*.csv" | sort
