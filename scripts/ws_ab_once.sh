set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "wsflat or WSFLAT or k12 or golden or kats or full_size or bad_launch or agree" > gpurun_out/ws_tests.log 2>&1
rc=$?; tail -5 gpurun_out/ws_tests.log; [ $rc -ne 0 ] && exit $rc
AB_WORKLOAD=mixed AB_ROUNDS=5 AB_VARIANTS="${WS_VARIANTS:-flat:8:0,wsflat:0x404:2,wsflat:0x404:3,wsflat:0x1408:2,wsflat:0x408:3,wsflat:0x204:3,wsflat:0x204:5,wsflat:0x208:4,wsflat:0x104:6,wsflat:0x104:8,wsflat:0x102:8}" timeout -k 10 200 python scripts/ab.py gpurun_out/ws_ab.json > gpurun_out/ws_ab.log 2>&1
rc=$?; tail -15 gpurun_out/ws_ab.log; exit $rc
