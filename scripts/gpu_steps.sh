#!/usr/bin/env bash
# One runner for the GPU box (through gpurun): each named step runs under its
# own time limit, output under gpurun_out/; the first step that fails (or
# faults, or times out) ends the script with its status.  Replaces round 3's
# single-use scripts/*_once.sh wrappers.
#
#   bash scripts/gpu_steps.sh STEP [STEP ...]
#
# Steps:
#   tests                 pytest -m gpu (one process, per-test timeout)
#   smoke                 __graft_entry__.smoke()
#   bench[:WL]            the default bench line (WL: tcp1500 | tcp9000 | mixed)
#   e2e[:WL]              the bench line with its host-resident (PCIe-inclusive) rates and small-batch latency
#   frames                the mixed bench line with its device frame-call diag (TX fill, RX verify)
#   crossover             bench.py --crossover: host calls at n = 1..256K on both sides of the CPU/GPU threshold
#   crossover_t1          the same with LVLIP_GATHER_THREADS=1 (the gather on the calling thread)
#   compose               scripts/compose_timing.py: level-ip's own stack per burst / flush, batched and not
#   dispatch              the round-6 dispatch, failure and composition GPU tests alone
#   rehearse:N            bench.py --gpus N self-launched over gloo, the ranks sharing the one GPU
#   rehearse_strong:N     the same with --workload tcp1500x64m (64M packets split over the N ranks)
#   rehearse_root:N       the same with --origin root (the batch scattered from rank 0's GPU first)
#   numa                  scripts/lab_numa.py (XCD <-> address-class locality probe)
#   window:SET            scripts/lab_window.py with LAB_SET=SET (read-order probes)
#   evidence:WL           scripts/evidence.sh for WL (bench + trace + PMC of the kernel AUTO runs)
#   pmc:WL                the PMC passes of that evidence alone (scripts/profile.sh)
#   ab:WL:VARIANTS        scripts/ab.py on WL with a variant list (AB_VARIANTS syntax, no ':' inside
#                         a variant here: use AB_VARIANTS directly for those)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r06}

run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($secs s): $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -25 "gpurun_out/$name.log"
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}

for step in "$@"; do
  case "$step" in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python bench.py ;;
    bench:*) wl=${step#bench:}; run "bench_$wl" 300 python bench.py --workload "$wl" ;;
    e2e) run e2e_tcp1500 300 python bench.py --e2e ;;
    e2e:*) wl=${step#e2e:}; run "e2e_$wl" 300 python bench.py --workload "$wl" --e2e ;;
    frames) run frames 600 python bench.py --workload mixed --frames ;;
    rehearse:*) n=${step#rehearse:}; run "rehearse_n$n" 300 env LVLIP_DIST_BACKEND=gloo python bench.py --gpus "$n" --steps 50 --warmup 10 ;;
    rehearse_strong:*) n=${step#rehearse_strong:}; run "rehearse_strong_n$n" 400 env LVLIP_DIST_BACKEND=gloo python bench.py --gpus "$n" --workload tcp1500x64m --steps 20 --warmup 5 ;;
    rehearse_root:*) n=${step#rehearse_root:}; run "rehearse_root_n$n" 300 env LVLIP_DIST_BACKEND=gloo python bench.py --gpus "$n" --origin root --steps 50 --warmup 10 ;;
    crossover) run crossover 600 python bench.py --crossover --steps 5 --warmup 2 --no-cpu-baseline ;;
    crossover_t1) run crossover_t1 600 env LVLIP_GATHER_THREADS=1 python bench.py --crossover --steps 5 --warmup 2 \
                    --no-cpu-baseline ;;
    compose) run compose 900 sh -c "python scripts/compose_timing.py > gpurun_out/${TAG}_compose.json" ;;
    dispatch) run dispatch 900 python -u -m pytest tests/test_dispatch_gpu.py tests/test_ref_tx_batch.py \
                tests/test_ref_rx_batch.py tests/test_ref_scale.py tests/test_skb_gpu.py tests/test_skb_list.py \
                tests/test_sanitize_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    numa) run numa 300 python scripts/lab_numa.py "gpurun_out/${TAG}_numa.json" ;;
    window:*) set_=${step#window:}; run "window_$set_" 400 env LAB_SET="$set_" python scripts/lab_window.py "gpurun_out/${TAG}_window_$set_.json" ;;
    evidence:*|pmc:*)
      wl=${step#*:}
      case "$wl" in mixed) kre=k_flat2 ;; *) kre=k_window ;; esac  # the kernel AUTO runs (bench.py KERNEL_FN)
      if [ "${step%%:*}" = evidence ]; then
        run "evidence_$wl" 900 env TAG="$TAG" WL="$wl" KRE="$kre" bash scripts/evidence.sh
      else  # the PMC passes alone, into the same evidence directory
        run "pmc_$wl" 600 env OUT="gpurun_out/evidence_${TAG}_$wl/prof" KRE="$kre" \
          BENCH="bench.py --workload $wl --steps 20 --warmup 3 --settle-ms 0 --no-cpu-baseline" bash scripts/profile.sh
      fi ;;
    ab:*) IFS=: read -r _ wl vars <<< "$step"
      run "ab_$wl" 600 env AB_WORKLOAD="$wl" AB_VARIANTS="$vars" python scripts/ab.py "gpurun_out/${TAG}_ab_$wl.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps ok: $*"
