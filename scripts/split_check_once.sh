set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local rc; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "full_size or config5 or max_int or max_batch or relaunch or auto_small" > gpurun_out/split_tests.log 2>&1
tail -3 gpurun_out/split_tests.log
AB_WORKLOAD=tcp1500x64m AB_SETTLE=30 AB_ROUNDS=3 AB_VARIANTS="auto:0:0,split64/auto:0:0" step timeout -k 10 300 python scripts/ab.py gpurun_out/split2_64m.json > gpurun_out/split2_64m.log 2>&1
tail -3 gpurun_out/split2_64m.log
AB_WORKLOAD=tcp9000 AB_ROUNDS=5 AB_VARIANTS="auto:0:0,window:0x302:8" step timeout -k 10 300 python scripts/ab.py gpurun_out/split2_9000.json > gpurun_out/split2_9000.log 2>&1
tail -3 gpurun_out/split2_9000.log
