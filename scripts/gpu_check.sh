#!/usr/bin/env bash
# One GPU session: GPU tests, then the bench (+ kernel sweep), each under its own
# time limit.  A test failure (rc 1) still lets the bench run; a crash, abort,
# fault or timeout (any other rc) stops the script so nothing else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---sweep --e2e} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json; tail -30 gpurun_out/bench.err
echo "pytest rc=$rc bench rc=$brc"
exit $(( rc > brc ? rc : brc ))
