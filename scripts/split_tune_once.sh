set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local rc; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
AB_WORKLOAD=tcp9000 AB_ROUNDS=5 AB_VARIANTS="window:0x302:8:0,split2/window:0x302:8:0,split3/window:0x302:8:0,split4/window:0x302:8:0,split6/window:0x302:8:0" step timeout -k 10 300 python scripts/ab.py gpurun_out/split3_9000.json > gpurun_out/split3_9000.log 2>&1
tail -5 gpurun_out/split3_9000.log
AB_WORKLOAD=tcp1500 AB_N=8388608 AB_SETTLE=60 AB_ROUNDS=5 AB_VARIANTS="window:0x402:12:0,split4/window:0x402:12:0,split6/window:0x402:12:0,split8/window:0x402:12:0,split12/window:0x402:12:0" step timeout -k 10 300 python scripts/ab.py gpurun_out/split3_8m.json > gpurun_out/split3_8m.log 2>&1
tail -5 gpurun_out/split3_8m.log
AB_WORKLOAD=tcp1500x64m AB_SETTLE=30 AB_ROUNDS=3 AB_VARIANTS="split32/window:0x402:12:0,split48/window:0x402:12:0,split64/window:0x402:12:0,split96/window:0x402:12:0" step timeout -k 10 300 python scripts/ab.py gpurun_out/split3_64m.json > gpurun_out/split3_64m.log 2>&1
tail -4 gpurun_out/split3_64m.log
