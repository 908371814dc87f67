#!/usr/bin/env bash
# PMC passes (one counter group per rocprofv3 run) over a short A/B run of two
# or more kernel variants on one workload (GPU box):
#   WL=mixed VARIANTS="flat:8:0,rflat:0x2004:12" KRE="k_flat2|k_rflat" bash scripts/pmc_ab.sh
# Outputs under gpurun_out/pmc_ab/<pass>/; every pass has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_ab}
mkdir -p $OUT
run() {
  local name=$1; shift
  AB_WORKLOAD=${WL:-mixed} AB_ROUNDS=1 AB_VARIANTS="$VARIANTS" timeout -s KILL ${PT:-120} \
    /opt/rocm/bin/rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 scripts/ab.py > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"; tail -3 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run trace --kernel-trace --stats
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$KRE"
run sq2 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT --kernel-include-regex "$KRE"
run fetch --pmc FETCH_SIZE --kernel-include-regex "$KRE"
python3 - "$OUT" "$KRE" <<'PY'
import csv, os, re, sys
from collections import defaultdict
out, kre = sys.argv[1], sys.argv[2]
agg = defaultdict(lambda: defaultdict(list))
for sub in ("sq", "sq2", "fetch"):
    p = os.path.join(out, sub, f"{sub}_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        name = r["Kernel_Name"]
        k = re.search(r"(k_\w+?)<[^>]*>|(k_\w+)", name)
        key = name.split("(")[0][-60:]
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    print(k)
    for n, v in sorted(c.items()):
        print(f"   {n:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
PY
