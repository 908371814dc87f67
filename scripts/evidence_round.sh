#!/usr/bin/env bash
# A round's GPU evidence in one call: the -m gpu suite, smoke(), then per config
# the default bench line, its rocprofv3 kernel trace and PMC passes
# (scripts/evidence.sh).  The first failing step stops everything.
#   TAG=r03 bash scripts/evidence_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
step() { local rc; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
if [ -z "${SKIP_TESTS:-}" ]; then
  step timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu_${TAG}.log 2>&1
  tail -2 gpurun_out/pytest_gpu_${TAG}.log
  step timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
  tail -1 gpurun_out/smoke_${TAG}.log
fi
for spec in ${CONFIGS:-tcp1500:k_window tcp9000:k_window mixed:k_flat2}; do
  wl=${spec%%:*}; kre=${spec##*:}
  TAG=$TAG WL=$wl KRE=$kre step bash scripts/evidence.sh
  head -c 400 gpurun_out/evidence_${TAG}_${wl}/bench.json; echo
done
