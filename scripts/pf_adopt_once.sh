# The product with k_flat2's descriptor prefetch against the previous revision
# (scripts/build_ab.sh HEAD~ -> level-ip_amd/ab/liblvlip_csum_ab.so) on mixed
# and on small-packet batches, in one process; the parity suite first.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pf_tests.log 2>&1
rc=$?; tail -2 gpurun_out/pf_tests.log; [ $rc -ne 0 ] && exit $rc
AB_ALT_LIB=level-ip_amd/ab/liblvlip_csum_ab.so AB_WORKLOAD=mixed AB_ROUNDS=11 \
  AB_VARIANTS="auto:0:0,alt/auto:0:0,flat:8:0,alt/flat:8:0" timeout -k 10 240 python scripts/ab.py gpurun_out/pf_adopt_mixed.json > gpurun_out/pf_adopt_mixed.log 2>&1
rc=$?; tail -5 gpurun_out/pf_adopt_mixed.log; [ $rc -ne 0 ] && exit $rc
exit 0
