#!/usr/bin/env bash
# A/B of the data-load cache policy for the AUTO kernel (LVLIP_LOAD_POLICY),
# interleaved in fresh processes.  POLICIES / WORKLOADS override the sets.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rnd in 1 2; do
  for w in ${WORKLOADS:-tcp1500 mixed tcp9000}; do
    for pol in ${POLICIES:-nt temporal}; do
      LVLIP_LOAD_POLICY=$pol timeout -k 10 240 python bench.py --workload $w --steps 100 --warmup 20 --no-cpu-baseline --no-verify \
        > gpurun_out/ab/$w.$pol.$rnd.json 2> gpurun_out/ab/$w.$pol.$rnd.err || exit $?
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'])" gpurun_out/ab/$w.$pol.$rnd.json $w $pol
    done
  done
done
