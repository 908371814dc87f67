# The mixed line's two modes against the address-translation counters (GPU box):
# six processes, each the mixed bench under one PMC pass (UTCL1 requests, hits,
# misses; UTCL2 busy) plus the kernel trace, so each process's mode shows in
# its own k_flat2 durations and counters.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/tlb_modes
mkdir -p $D
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 /opt/rocm/bin/rocprofv3 --kernel-trace --stats \
      --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_PERMISSION_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE \
      --output-format csv -d $D/p$i -o p -- python3 bench.py --workload mixed --steps 60 --warmup 5 --no-cpu-baseline \
      > $D/p$i.json 2> $D/p$i.err
  rc=$?; if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; tail -5 $D/p$i.err; exit $rc; fi
  python3 - $D/p$i <<'PY'
import csv, glob, json, sys, statistics as st
d = sys.argv[1]
line = json.loads(open(d + ".json").read().strip().splitlines()[-1])
agg = {}
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_flat2" in r["Kernel_Name"]:
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
dur = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_flat2" in r["Kernel_Name"]:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(d, "line", line["value"], "kernel_ms", line["roofline"]["kernel_ms"], "trace median us",
      round(st.median(dur), 1) if dur else None,
      {k: round(st.median(v)) for k, v in sorted(agg.items())}, flush=True)
PY
done
