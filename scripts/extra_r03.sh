#!/usr/bin/env bash
# Round-3 extras on one GPU: configs[4]'s 64M x 1500 B batch (96 GB) on one GPU,
# and the self-launched N = 2 / 4 path rehearsed over gloo on the one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local rc; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python bench.py --workload tcp1500x64m --steps 100 --warmup 20 --no-cpu-baseline \
    > gpurun_out/r03_bench_64m.json 2> gpurun_out/r03_bench_64m.err
head -c 600 gpurun_out/r03_bench_64m.json; echo
for n in 2 4; do
  LVLIP_DIST_BACKEND=gloo step timeout -k 10 240 python bench.py --gpus $n \
      > gpurun_out/r03_bench_n${n}_selflaunch.json 2> gpurun_out/r03_bench_n${n}_selflaunch.err
  head -c 300 gpurun_out/r03_bench_n${n}_selflaunch.json; echo
done
