set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_WORKLOAD=tcp1500x64m AB_SETTLE=30 AB_ROUNDS=3 AB_VARIANTS="auto:0:0,split4/auto:0:0,split16/auto:0:0,split64/auto:0:0,split256/auto:0:0" timeout -k 10 300 python scripts/ab.py gpurun_out/split_64m.json > gpurun_out/split_64m.log 2>&1
rc=$?; tail -6 gpurun_out/split_64m.log; [ $rc -ne 0 ] && exit $rc
AB_WORKLOAD=tcp1500 AB_N=8388608 AB_SETTLE=60 AB_ROUNDS=3 AB_VARIANTS="auto:0:0,split2/auto:0:0,split4/auto:0:0,split8/auto:0:0" timeout -k 10 300 python scripts/ab.py gpurun_out/split_8m.json > gpurun_out/split_8m.log 2>&1
rc=$?; tail -5 gpurun_out/split_8m.log; exit $rc
