#!/usr/bin/env bash
# Read-request size mix at the L2/fabric boundary (calibrates the FETCH_SIZE x2
# rule): one PMC pass per workload, every kernel of the bench command, counters
# only (no trace domains beside them).  Output: gpurun_out/tcc/<workload>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for w in ${WORKLOADS:-tcp1500 mixed}; do
  OUT=gpurun_out/tcc/$w
  mkdir -p $OUT
  timeout -k 10 ${PROF_TIMEOUT:-240} /opt/rocm/bin/rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum \
      -T --output-format csv -d $OUT -o tcc -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-verify > $OUT/log 2>&1
  rc=$?
  echo "pass $w rc=$rc"; tail -2 $OUT/log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
