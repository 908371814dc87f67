# k_window_dyn (lab id 15): parity subset, then A/B against AUTO on tcp1500 and
# tcp9000 (7 rounds in one process each), then its per-wave stamps.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/dyn
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "golden or kats or configs_small or full_size or alignment" > gpurun_out/dyn/par.log 2>&1
rc=$?; tail -2 gpurun_out/dyn/par.log; [ $rc -ne 0 ] && exit $rc
for wl in tcp1500 tcp9000; do
  AB_WORKLOAD=$wl AB_ROUNDS=7 AB_VARIANTS="${DYN_VARIANTS:-auto:0:0,window_dyn:0x402:12,window_dyn:0x402:8,window_dyn:0x202:12,window_dyn:0x202:8,window_dyn:0x102:12}" timeout -k 10 240 python scripts/ab.py gpurun_out/dyn/ab_$wl.json > gpurun_out/dyn/ab_$wl.log 2>&1
  rc=$?; grep GB/s gpurun_out/dyn/ab_$wl.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/dyn/ab_$wl.log; exit $rc; }
done
TAIL_DYN=1 timeout -k 10 120 python scripts/lab_tail.py gpurun_out/dyn/tail_dyn12.json 12 12 > gpurun_out/dyn/tail.log 2>&1
rc=$?; tail -1 gpurun_out/dyn/tail.log; exit $rc
