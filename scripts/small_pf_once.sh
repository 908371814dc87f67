# k_flat2's descriptor prefetch on uniform small-segment batches (U 4, the
# shape AUTO runs below 320 B, and U 8), ~1.6 GB each, against the product.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or kats" > gpurun_out/spf_tests.log 2>&1
rc=$?; tail -1 gpurun_out/spf_tests.log; [ $rc -ne 0 ] && exit $rc
for wl in ${SPF_WLS:-tcp64 tcp128 tcp256 tcp512}; do
  AB_WORKLOAD=$wl AB_ROUNDS=7 AB_VARIANTS="auto:0:0,flat:4:0,flat_occ:0x804:0,flat_occ:0x4704:0,flat:8:0" \
    timeout -k 10 200 python scripts/ab.py gpurun_out/spf_$wl.json 2>&1 | grep -v amdgpu.ids
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
