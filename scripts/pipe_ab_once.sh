set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "golden or kats or full_size or bad_launch or alignment_length or configs_small or empty_and_tiny" > gpurun_out/pipe_tests.log 2>&1
rc=$?; tail -4 gpurun_out/pipe_tests.log; [ $rc -ne 0 ] && exit $rc
AB_WORKLOAD=mixed AB_ROUNDS=7 AB_VARIANTS="flat:8:0,flat:0x808:0,flat:0x806:0,flat:0x804:0,flat:0x802:0,flat:4:0" timeout -k 10 200 python scripts/ab.py gpurun_out/pipe_ab.json > gpurun_out/pipe_ab.log 2>&1
rc=$?; tail -8 gpurun_out/pipe_ab.log; exit $rc
