#!/usr/bin/env bash
# One GPU session: GPU tests, then the bench (+ kernel sweep), each under its own
# time limit.  Any test failure stops the script, so after a fault nothing else
# touches the GPU in the same call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping before the bench (a failed GPU test may be a fault)"; exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---sweep --e2e} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json; tail -30 gpurun_out/bench.err
echo "pytest rc=$rc bench rc=$brc"
exit $(( rc > brc ? rc : brc ))
