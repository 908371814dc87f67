# k_flat2 U 8 with s_setprio around the sweep's load issue / phase 1 (lab id
# 13, Q << 16) against the product on mixed, 9 rounds in one process.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_WORKLOAD=mixed AB_ROUNDS=9 AB_VARIANTS="${PRIO_VARIANTS:-auto:0:0,flat_occ:0x4508:0,flat_occ:0x84508:0,flat_occ:0xA4508:0,flat_occ:0x24508:0}" timeout -k 10 240 python scripts/ab.py gpurun_out/prio_ab.json > gpurun_out/prio_ab.log 2>&1
rc=$?; tail -8 gpurun_out/prio_ab.log; exit $rc
