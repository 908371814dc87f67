#!/usr/bin/env bash
# One GPU session for a round's checkpoint: the -m gpu suite, smoke(), then the
# default bench line (configs[1]), each under its own time limit; the first
# failure stops the script, so after a fault nothing else touches the GPU.
#   bash scripts/gpu_round.sh [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local rc; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 ${PYTEST_TIMEOUT:-420} python -u -m pytest tests -m gpu -x -v --timeout 120 \
    --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
tail -3 gpurun_out/pytest_gpu.log
step timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
step timeout -k 10 240 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
