set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "rflat or golden or kats or full_size or bad_launch" > gpurun_out/rf_tests.log 2>&1
rc=$?; tail -5 gpurun_out/rf_tests.log; [ $rc -ne 0 ] && exit $rc
AB_WORKLOAD=mixed AB_ROUNDS=5 AB_VARIANTS="flat:8:0,rflat:0x1004:12,rflat:0x1004:8,rflat:0x1008:8,rflat:0x1006:12,rflat:0x2004:12,rflat:0x2008:8,rflat:0x1002:16,rflat:0x1004:16" timeout -k 10 200 python scripts/ab.py gpurun_out/rf_ab.json > gpurun_out/rf_ab.log 2>&1
rc=$?; tail -15 gpurun_out/rf_ab.log; exit $rc
