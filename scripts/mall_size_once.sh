# Does k_flat2 run faster when its batch is resident in the MALL (256 MB
# Infinity Cache)?  The mixed batch at 2M / 256K / 128K / 64K frames, k_window
# on MTU batches of the same byte sizes, back-to-back launches (the premise of
# a data prefetch into the MALL).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 2097152 262144 131072 65536; do
  AB_N=$n AB_WORKLOAD=mixed AB_ROUNDS=5 AB_VARIANTS="flat:8:0" timeout -k 10 120 python scripts/ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/n=$n /"
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
for n in 1048576 131072 65536 32768; do
  AB_N=$n AB_WORKLOAD=tcp1500 AB_ROUNDS=5 AB_VARIANTS="auto:0:0" timeout -k 10 120 python scripts/ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/n=$n /"
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
