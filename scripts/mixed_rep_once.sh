# Run-to-run spread of the mixed bench line against its kernel trace (GPU box):
# bench, trace, bench, bench; one process each.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/mixed_rep
mkdir -p $D
step() { local rc; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 180 python3 bench.py --workload mixed --no-cpu-baseline > $D/b1.json 2> $D/b1.err
step timeout -k 10 240 /opt/rocm/bin/rocprofv3 --kernel-trace --stats -T --output-format csv \
    -d $D/trace -o trace -- python3 bench.py --workload mixed --no-cpu-baseline > $D/t.json 2> $D/t.err
step timeout -k 10 180 python3 bench.py --workload mixed --no-cpu-baseline > $D/b2.json 2> $D/b2.err
step timeout -k 10 180 python3 bench.py --workload mixed --no-cpu-baseline > $D/b3.json 2> $D/b3.err
for f in b1 t b2 b3; do python3 -c "
import json; l=json.loads(open('$D/$f.json').read().strip().splitlines()[-1]); print('$f', l['value'], l['roofline']['kernel_ms'], l['dist']['ranks'][0]['pci'])"; done
grep k_flat2 $D/trace/trace_kernel_stats.csv | cut -d, -f1-4
