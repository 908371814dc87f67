# FETCH_SIZE and L2 hits of k_flat2 with and without the descriptor prefetch
# (lab id 13, P x 640 tiles ahead) on mixed, one counter group per pass.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/pf_pmc
mkdir -p $OUT
run() {
  local name=$1; shift
  AB_WORKLOAD=mixed AB_ROUNDS=1 AB_VARIANTS="flat:8:0,flat_occ:0x4508:0" timeout -s KILL 120 \
    /opt/rocm/bin/rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 scripts/ab.py > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 $OUT/$name.log; exit $rc; fi
}
run fetch --pmc FETCH_SIZE --kernel-include-regex k_flat2
run tcc --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_flat2
run tcc2 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex k_flat2
python3 - $OUT <<'PY'
import csv, os, sys
from collections import defaultdict
out = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for sub in ("fetch", "tcc", "tcc2"):
    p = os.path.join(out, sub, f"{sub}_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        agg[r["Kernel_Name"].split("(")[0][-70:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    print(k)
    for n, v in sorted(c.items()):
        print(f"   {n:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
PY
