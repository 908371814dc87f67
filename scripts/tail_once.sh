# lab_tail.py: k_window's per-wave end times at 12 waves/CU in workgroups of
# 4, 8 and 12 waves (one process each).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/tail
export TMPDIR=/tmp
for spec in ${TAIL_SPECS:-12:4 12:12 12:4 12:12 8:8 8:4}; do
  w=${spec%%:*}; p=${spec##*:}
  timeout -k 10 120 python scripts/lab_tail.py gpurun_out/tail/w${w}_p${p}_$RANDOM.json $w $p > gpurun_out/tail/last.log 2>&1
  rc=$?; tail -1 gpurun_out/tail/last.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/tail/last.log; exit $rc; }
done
exit 0
