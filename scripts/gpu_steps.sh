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
#   txstore               scripts/lab_tx_store.py (TX field-store A/B + probes)
#   fhost[:R]             scripts/lab_frames_host.py (host frame pipeline: ramps, threads; R rounds)
#   rehearse:N            bench.py --gpus N self-launched over gloo, the ranks sharing the one GPU
#   rehearse_strong:N     the same with --workload tcp1500x64m (64M packets split over the N ranks)
#   rehearse_root:N       the same with --origin root (the batch scattered from rank 0's GPU first)
#   wb                    scripts/lab_wb.py (field-store forms paired with the RX + L4 sweep)
#   txpmc                 FETCH_SIZE / WRITE_SIZE passes of the TX variants
#   modes:K               K processes of scripts/lab_modes.py (mixed line modes)
#   numa                  scripts/lab_numa.py (XCD <-> address-class locality probe)
#   cputh, cputh_spin     scripts/lab_cpu_threads.py (host CPU time of the frame calls per thread;
#                         _spin: LVLIP_BLOCK_MIN=0)
#   window:SET            scripts/lab_window.py with LAB_SET=SET (read-order probes)
#   evidence:WL           scripts/evidence.sh for WL (bench + trace + PMC of the kernel AUTO runs)
#   pmc:WL                the PMC passes of that evidence alone (scripts/profile.sh)
#   ab:WL:VARIANTS        scripts/ab.py on WL with a variant list (AB_VARIANTS syntax, no ':' inside
#                         a variant here: use AB_VARIANTS directly for those)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05}

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
    frames) run frames 300 python bench.py --workload mixed --frames ;;
    rehearse:*) n=${step#rehearse:}; run "rehearse_n$n" 300 env LVLIP_DIST_BACKEND=gloo python bench.py --gpus "$n" --steps 50 --warmup 10 ;;
    rehearse_strong:*) n=${step#rehearse_strong:}; run "rehearse_strong_n$n" 400 env LVLIP_DIST_BACKEND=gloo python bench.py --gpus "$n" --workload tcp1500x64m --steps 20 --warmup 5 ;;
    rehearse_root:*) n=${step#rehearse_root:}; run "rehearse_root_n$n" 300 env LVLIP_DIST_BACKEND=gloo python bench.py --gpus "$n" --origin root --steps 50 --warmup 10 ;;
    wb) run wb 400 python scripts/lab_wb.py "gpurun_out/${TAG}_wb.json" 5 ;;
    fhost) run fhost 500 python scripts/lab_frames_host.py "gpurun_out/${TAG}_frames_host.json" 3 ;;
    fhost:*) r=${step#fhost:}; run fhost 500 python scripts/lab_frames_host.py "gpurun_out/${TAG}_frames_host.json" "$r" ;;
    txstore) run txstore 400 python scripts/lab_tx_store.py "gpurun_out/${TAG}_tx_store.json" 7 ;;
    txpmc)
      for v in ${TXPMC_VARIANTS:-tx_product tx_nt tx_sec32 rx_l4}; do
        for c in FETCH_SIZE WRITE_SIZE; do
          run "txpmc_${v}_$c" 180 /opt/rocm/bin/rocprofv3 --pmc "$c" --kernel-include-regex "k_flat2|k_probe" \
            --output-format csv -d "gpurun_out/txpmc/${v}_$c" -o "${v}_$c" -- python3 scripts/lab_tx_store.py --only "$v" 20
        done
      done
      run txtrace 180 /opt/rocm/bin/rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/txpmc/trace \
        -o trace -- python3 scripts/lab_tx_store.py --only tx_product 20 ;;
    numa) run numa 300 python scripts/lab_numa.py "gpurun_out/${TAG}_numa.json" ;;
    cputh) run cputh 300 python scripts/lab_cpu_threads.py "gpurun_out/${TAG}_cpu_threads.json" 40 ;;
    cputh_spin) run cputh_spin 300 env LVLIP_BLOCK_MIN=0 python scripts/lab_cpu_threads.py "gpurun_out/${TAG}_cpu_threads_spin.json" 40 ;;
    window:*) set_=${step#window:}; run "window_$set_" 400 env LAB_SET="$set_" python scripts/lab_window.py "gpurun_out/${TAG}_window_$set_.json" ;;
    modes:*)
      k=${step#modes:}
      for i in $(seq 1 "$k"); do run "modes_p$i" 240 python scripts/lab_modes.py "gpurun_out/${TAG}_modes_p$i.json"; done ;;
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
