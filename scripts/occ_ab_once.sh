set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "golden or kats or full_size or bad_launch or agree" > gpurun_out/occ_tests.log 2>&1
rc=$?; tail -3 gpurun_out/occ_tests.log; [ $rc -ne 0 ] && exit $rc
AB_WORKLOAD=mixed AB_ROUNDS=7 AB_VARIANTS="${OCC_VARIANTS:-flat:8:0,flat_occ:0x508:0,flat_occ:0x1508:0,flat_occ:0x608:0,flat_occ:0x1608:0,flat_occ:0x706:0,flat_occ:0x1706:0,flat:6:0}" timeout -k 10 200 python scripts/ab.py gpurun_out/occ_ab.json > gpurun_out/occ_ab.log 2>&1
rc=$?; tail -12 gpurun_out/occ_ab.log; exit $rc
