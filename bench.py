#!/usr/bin/env python3
"""bench.py — device-resident Internet-checksum throughput on MI355X.

One step = one lvlip_csum_batch_dev launch over one synthetic batch already
resident in HBM (BASELINE.json configs[1] by default: 1 M x 1500 B TCP
segments).  Prints ONE JSON line (rank 0):

  value       whole-job GB/s = sum over ranks of algorithmic bytes x K / max-over-ranks time
  roofline    the checksum kernel's achieved algorithmic GB/s (HIP events on the launch
              stream) against the 8 TB/s HBM3E peak; frac_aggregate = value / (N x 8 TB/s);
              traffic = PMC-measured HBM bytes per launch from profiles/ when a matching
              measurement is committed (traffic_source names the file: the builder's
              box, not this run's), else null; achieved_contract / frac_contract
              count SURVEY.md §8(d)'s algorithmic bytes exactly (the bytes summed +
              2 B per result; achieved counts the summed bytes only, 0.13 % less)
  verified_bit_exact  every one of the N outputs of the timed batch, copied back from
              HBM after the timed loop, equals level-ip's own checksum() (oracle/_ref,
              compiled from src/utils.c) run over the same bytes; on every rank
  cpu_baseline  that reference checksum() on the host cores (rank 0, N=1): all
              cores of the process's affinity mask over the whole timed batch, plus
              one-core and 16-thread figures

Before the W warm-up steps every rank runs untimed steps for --settle-ms of wall
time (default 250 ms), so the timed region starts at the GPU's sustained clocks
rather than in its ramp from idle (diag.settle).

Multi-GPU (BASELINE configs[4]): `python bench.py --gpus N` starts
its N ranks itself, one process per GPU, before anything in the parent touches
the GPU; under `python -m torch.distributed.run --nproc-per-node N bench.py --gpus
N` the launcher's ranks are used instead (WORLD_SIZE must equal N).  Every rank
checksums its own shard (packets rank*n .. rank*n+n-1 of the stream: weak
scaling, no collective on the data path); RCCL carries only the barriers, the
max-over-ranks time and the per-rank report.  Under RCCL every rank must own a
distinct GPU (checked by PCI bus id); LVLIP_DIST_BACKEND=gloo rehearses several
ranks on one GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # checker + cpu_baseline leg only (pyoracle)

import numpy as np  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "device-resident checksum GB/s over packet batch; % of HBM-read roofline"
WORKLOAD_TEXT = {
    "tcp1500": "1M x 1500 B TCP segments (MTU), pseudo-header + payload checksum, "
               "16-B aligned slots (stride 1504)",
    "tcp9000": "1M x 9000 B TCP segments (jumbo), pseudo-header + payload checksum, "
               "16-B aligned slots (stride 9008)",
    "mixed": "2M frames: 20 B IPv4 headers + 64-1460 B ICMP/TCP payloads interleaved "
             "(4M descriptors, skb offsets 14/34)",
    "tcp1500x64m": "64M x 1500 B TCP segments (96 GB) split over the ranks (strong scaling), "
                   "16-B aligned slots (stride 1504)",
}
STRONG = {"tcp1500x64m": 64 << 20}  # workload -> total packets over all ranks
VERIFY_SPAN = 2 << 30  # host bytes per verification chunk (copied back from HBM)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs = ranks on this node (default: WORLD_SIZE, else 1).  N > 1 "
                        "without a torch.distributed launcher: bench.py starts the N ranks")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--settle-ms", type=float, default=250.0,
                   help="untimed steps before the warm-up until this much wall time has "
                        "passed (GPU clock ramp from idle; 0 disables)")
    p.add_argument("--workload", default="tcp1500", choices=sorted(WORKLOAD_TEXT))
    p.add_argument("--n", "--packets", dest="n", type=int, default=None,
                   help="packets (frames for mixed) per rank (--packets under torch.distributed.run, "
                        "whose own parser takes --n for a prefix of its options)")
    p.add_argument("--kernel", default="auto",
                   choices=["auto", "wave", "flat", "window", "wflat", "lane"])
    p.add_argument("--unroll", type=int, default=0)
    p.add_argument("--waves-per-cu", type=int, default=0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--dry-run", action="store_true",
                   help="rehearse the launch / rendezvous / report path on the CPU (gloo, no "
                        "GPU work, small batch): the line carries dry_run=true and no throughput")
    p.add_argument("--sweep", action="store_true", help="also time every kernel variant (stderr)")
    p.add_argument("--frames", action="store_true",
                   help="diag: device-resident frame batches (TX fill, RX verify) on the mixed frames")
    p.add_argument("--origin", choices=["local", "root"], default="local",
                   help="root: the whole batch starts on rank 0's GPU and is scattered "
                        "point to point first (timed separately, diag.scatter)")
    p.add_argument("--crossover", action="store_true",
                   help="diag: host calls at n = 1..256K frames on both sides of the CPU/GPU threshold "
                        "(lvlip_csum_ctx_set_cpu_max), wall and CPU time per call")
    p.add_argument("--no-crossover", action="store_true",
                   help="with --frames: leave the crossover curve out (kernel traces of the frame calls)")
    p.add_argument("--e2e", action="store_true",
                   help="also time the host-resident path (PCIe-inclusive; stderr + diag)")
    return p.parse_args(argv)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# the device function each --kernel choice runs (what the PMC records name)
KERNEL_FN = {"window": "k_window", "wave": "k_stream", "flat": "k_flat2", "wflat": "k_wflat",
             "lane": "k_lane"}


def traffic_from_profiles(workload: str, kernel_label: str, kernel_fn: str):
    """(HBM bytes per launch, file) measured by rocprofv3 PMC (profiles/*pmc*.json,
    see profiles/README.md) for this workload, launch label and device function
    (the newest file wins), or None when no matching measurement is committed.
    The counters are the builder's box's, committed with the code: the bench
    does not run a PMC pass itself (it would need rocprofv3 around it)."""
    pdir = os.path.join(ROOT, "profiles")
    best = None
    if not os.path.isdir(pdir):
        return None
    for fn in sorted(os.listdir(pdir)):
        if not (fn.endswith(".json") and "pmc" in fn):
            continue
        try:
            with open(os.path.join(pdir, fn)) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        kernels = rec.get("kernels") if isinstance(rec, dict) else None
        if not isinstance(kernels, list):  # other PMC summaries (frames, lane) have other shapes
            continue
        for r in kernels:
            if not isinstance(r, dict):
                continue
            if (r.get("workload") == workload and r.get("kernel") == kernel_label
                    and r.get("kernel_regex") == kernel_fn):
                best = (r.get("hbm_bytes_per_launch"), f"profiles/{fn}")
    return best


# ------------------------------------------------------------------ host CPUs --

def host_cpus() -> dict:
    """What the host offers this process: the affinity mask (what threads can
    run on), os.cpu_count() (the machine) and the cgroup CPU quota, if any."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
        except (OSError, ValueError):
            pass
    return {"nproc": aff, "machine_cpus": os.cpu_count(), "cgroup_cpu_quota": quota,
            "cpu_model": _cpu_model()}


def usable_cpus(cpus: dict) -> int:
    """The CPUs this process may use: its affinity mask, limited by the cgroup
    CPU quota when one is set (the GPU box: 256 CPUs in the mask, a 16-CPU
    quota, where 256 threads run slower than 16)."""
    n = cpus["nproc"]
    if cpus["cgroup_cpu_quota"]:
        n = max(1, min(n, int(cpus["cgroup_cpu_quota"] + 0.999)))
    return n


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ------------------------------------------------------------- verification --

def _chunks(descs: np.ndarray, span_max: int):
    """Consecutive descriptor ranges [lo, hi) whose byte span is at most
    span_max (a single descriptor may exceed it), with the span's start."""
    n = descs.size
    off = descs["offset"].astype(np.uint64)
    end = off + np.maximum(descs["len"], 0).astype(np.uint64)
    lo = 0
    step = max(1, n)
    while lo < n:
        hi = min(n, lo + step)
        while True:
            a = int(off[lo:hi].min()) & ~15
            e = int(end[lo:hi].max())
            if e - a <= span_max or hi - lo == 1:
                break
            hi = lo + max(1, (hi - lo) // 2)
        step = max(hi - lo, 1)
        yield lo, hi, a, (e + 15) & ~15
        lo = hi


def verify_timed_batch(b, base, out, threads: int, keep_first: bool):
    """All outputs of the timed batch against level-ip's own checksum() over the
    same bytes, copied back from HBM after the timed loop (the checker: oracle/_ref,
    or the oracle restatement where the reference was not built).

    Returns (result dict, (host bytes, rebased descriptors) of the first chunk
    when keep_first, for the CPU baseline)."""
    import pyoracle  # test infrastructure: the checker

    use_ref = pyoracle.reflib() is not None
    got_all = out[: b.n].cpu().numpy().view(np.uint16)
    bad, ref_s, first = 0, 0.0, None
    for lo, hi, a, e in _chunks(b.descs, VERIFY_SPAN):
        host = base[a:e].cpu().numpy()
        d = b.descs[lo:hi].copy()
        d["offset"] -= np.uint64(a)
        t0 = time.perf_counter()
        want = pyoracle.batch(host, d, threads=threads, opt=0, use_reference=use_ref)
        ref_s += time.perf_counter() - t0
        bad += int(np.count_nonzero(want != got_all[lo:hi]))
        if keep_first and first is None:
            first = (host, d)
    return {"ok": bad == 0, "descriptors": b.n, "mismatches": bad,
            "checker": "reference" if use_ref else "port", "threads": threads,
            "checker_s": round(ref_s, 3)}, first


def cpu_baseline(b, first, cpus: dict, budget_s: float = 1.0):
    """level-ip's checksum() (oracle/_ref, -O0 as its Makefile builds it) on the
    host: every core of the affinity mask over the timed batch's bytes (its
    first <= 2 GiB, the whole batch for configs[1]), pthreads over contiguous
    packet ranges; plus 16 threads, one core, the same algorithm at -O2 and the
    product's own per-call drop-in on a 131 072-descriptor sample."""
    import pyoracle  # test infrastructure: the reported CPU baseline only

    import lvlip

    use_ref = pyoracle.reflib() is not None
    kind = "reference" if use_ref else "port"
    host, d = first
    nbytes = int(np.maximum(d["len"], 0).sum()) + 2 * d.size

    def rate(h, dd, thr, nb, budget, **kw):
        reps, t0 = 0, time.perf_counter()
        while True:
            pyoracle.batch(h, dd, threads=thr, **kw)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return nb * reps / dt / 1e9, reps, dt

    cores = usable_cpus(cpus)
    allc, reps, dt = rate(host, d, cores, nbytes, budget_s, opt=0, use_reference=use_ref)
    aff = None
    if cpus["nproc"] != cores:
        aff = rate(host, d, cpus["nproc"], nbytes, budget_s, opt=0, use_reference=use_ref)[0]
    # one-core figures on a sample (the same packets' first descriptors)
    ns = min(d.size, 131072)
    sd = d[:ns].copy()
    ea = int((sd["offset"] + np.maximum(sd["len"], 0).astype(np.uint64)).max())
    sh = host[: (ea + 15) & ~15]
    sb = int(np.maximum(sd["len"], 0).sum()) + 2 * ns
    one = rate(sh, sd, 1, sb, 2 * budget_s, opt=0, use_reference=use_ref)[0]
    o2 = rate(sh, sd, 1, sb, budget_s, opt=2)[0]
    dropin = rate(sh, sd, 1, sb, budget_s, csum_fn=lvlip.lib().checksum)[0]
    return {
        "value": round(allc, 3), "unit": "GB/s", "cores": cores, "kind": kind,
        "sample": (f"{d.size} descriptors / {nbytes / 1e6:.1f} MB of the timed {b.name} batch, "
                   f"copied back from HBM; {reps} passes in {dt:.2f} s on {cores} threads "
                   f"(pthreads over contiguous packet ranges, one per usable CPU: the affinity mask "
                   f"of {cpus['nproc']} CPUs under a cgroup quota of {cpus['cgroup_cpu_quota']}); "
                   f"level-ip {'src/utils.c compiled -O0 as its Makefile builds it' if use_ref else 'oracle restatement -O0'}"),
        "nproc": cpus["nproc"], "cores_used": cores, "machine_cpus": cpus["machine_cpus"],
        "cgroup_cpu_quota": cpus["cgroup_cpu_quota"], "cpu_model": cpus["cpu_model"],
        "affinity_threads_GBps": None if aff is None else round(aff, 3),
        "one_core_GBps": round(one, 3),
        "one_core_O2_restatement_GBps": round(o2, 3),
        "dropin_one_core_GBps": round(dropin, 3),
    }


# ------------------------------------------------------------------ launcher --

def self_launch(world: int) -> int:
    """`bench.py --gpus N` without a torch.distributed launcher: start the N
    ranks as child processes of this one (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* as torch.distributed.run sets them), one GPU each.  This process
    never touches the GPU (no torch import).  If a rank fails, the others are
    stopped (by PID) and the first failure's status is returned."""
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LVLIP_BENCH_LAUNCHER="bench.py")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc, live = 0, list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 1
                log(f"bench.py: rank {procs.index(p)} exited with status {r}; stopping the others")
                for q in live:
                    q.terminate()
        time.sleep(0.02)
    return rc


def main(argv=None):
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        world = args.gpus if args.gpus is not None else 1
        if world < 1:
            raise SystemExit("bench.py: --gpus must be >= 1")
        if world > 1:
            raise SystemExit(self_launch(world))
    else:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} "
                             "ranks; they must agree")
    run(args, world)


def _rank_info(torch, dev, rank: int, local: int) -> dict:
    info = {"rank": rank, "local_rank": local, "host": socket.gethostname()}
    if dev is not None and dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        info.update({"device": dev.index, "name": p.name,
                     "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
                     "uuid": str(getattr(p, "uuid", ""))})
    return info


def run(args, world: int):
    import torch
    import torch.distributed as dist

    import workloads

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    launcher = os.environ.get("LVLIP_BENCH_LAUNCHER") or ("torch.distributed.run" if world > 1 else None)
    # RCCL (backend "nccl") across the node's GPUs, one per rank;
    # LVLIP_DIST_BACKEND=gloo rehearses the N>1 code path with several ranks on
    # one GPU (device = local rank mod count); --dry-run has no GPU at all.
    backend = "gloo" if args.dry_run else os.environ.get("LVLIP_DIST_BACKEND", "nccl")
    dev = None
    if not args.dry_run:
        import lvlip

        ndev = torch.cuda.device_count()
        if ndev == 0 or lvlip.device_count() == 0:
            raise SystemExit(f"bench.py rank {rank}: needs a HIP device (none visible)")
        if backend == "nccl" and world > 1:
            if ndev < local_world:
                raise SystemExit(
                    f"bench.py rank {rank}: {local_world} ranks on this node need {local_world} GPUs "
                    f"(one per rank under RCCL), {ndev} visible; LVLIP_DIST_BACKEND=gloo rehearses "
                    "several ranks on one GPU")
            dev = torch.device("cuda", local)
        else:
            dev = torch.device("cuda", local % ndev)
        torch.cuda.set_device(dev)
    if world > 1:
        from datetime import timedelta

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=timedelta(minutes=10))
        else:
            dist.init_process_group(backend, timeout=timedelta(minutes=10))
    coll_dev = dev if backend == "nccl" and world > 1 else torch.device("cpu")

    ranks = [_rank_info(torch, dev, rank, local)]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, _rank_info(torch, dev, rank, local))
        if backend == "nccl":
            where = [(r["host"], r.get("pci")) for r in ranks]
            if len(set(where)) != world:
                raise SystemExit(f"bench.py rank {rank}: ranks share a GPU under RCCL: {where}")

    if args.workload in STRONG:
        # strong scaling: a fixed batch, contiguous packet ranges per rank
        total = args.n or STRONG[args.workload]
        first = total * rank // world
        n = total * (rank + 1) // world - first
    else:
        # weak scaling: each rank owns the next n packets of the stream
        n = args.n or (1 << 21 if args.workload == "mixed" else 1 << 20)
        first = rank * n
    if args.dry_run:
        n = min(n, 4096)
        first = rank * n
    scatter_diag = None
    if args.origin == "root" and world > 1 and not args.dry_run:
        import shard

        # the batch originates on one GPU; each rank receives its
        # byte-balanced shard point to point (RCCL over xGMI), timed on its own
        total_n = n * world if args.workload not in STRONG else (args.n or STRONG[args.workload])
        full, fdescs = None, None
        if rank == 0:
            fb = workloads.make(args.workload, n=total_n, first=0)
            fbase, _, _ = workloads.to_device(fb, dev)
            full = fbase if backend == "nccl" else fbase.cpu()
            fdescs = fb.descs
        dist.barrier()
        torch.cuda.synchronize(dev)
        ts = time.perf_counter()
        lbuf, ldescs, _ = shard.scatter_from_root(full, fdescs, coll_dev)
        torch.cuda.synchronize(dev)
        dist.barrier()
        t_sc = time.perf_counter() - ts
        sent = torch.tensor([float(lbuf.numel())], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(sent)
        scatter_diag = {"seconds": round(t_sc, 4), "bytes": int(sent[0]),
                        "GBps": round(float(sent[0]) / t_sc / 1e9, 2)}
        b = workloads.Batch(args.workload, ldescs, int(lbuf.numel()),
                            np.zeros(ldescs.size, np.uint8), 0,
                            int(np.maximum(ldescs["len"], 0).sum()))
        base = torch.zeros((lbuf.numel() + 15) // 16 * 16 + 16, dtype=torch.uint8, device=dev)
        base[: lbuf.numel()] = lbuf.to(dev)
        descs = torch.from_numpy(ldescs.view(np.uint8).copy()).to(dev)
        out = torch.empty(max(b.n, 1), dtype=torch.int16, device=dev)
        del full, lbuf
    else:
        b = workloads.make(args.workload, n=n, first=first)
        if args.dry_run:
            base = descs = out = None
        else:
            base, descs, out = workloads.to_device(b, dev)

    # the batch's average packet length, as a caller that built it knows it
    len_hint = b.algo_bytes // max(1, b.n)
    if args.dry_run:
        stream = None
        kernel = 0

        def step():
            pass

        def sync():
            pass
    else:
        import lvlip

        stream = torch.cuda.current_stream(dev)
        kernel = lvlip.KERNEL_NAMES[args.kernel]
        torch.cuda.synchronize(dev)

        def step():
            lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), stream.cuda_stream,
                            kernel, args.unroll, args.waves_per_cu, len_hint)

        def sync():
            torch.cuda.synchronize(dev)

    # Bring the GPU to its sustained clocks before the W warm-up steps: from idle,
    # the first ~15 ms of launches run 5-25 % slow (scripts/warm_curve.py,
    # DESIGN.md §5), which a 5+20-step run would otherwise time.  Untimed, and
    # reported in diag.settle.  With N > 1 ranks the first collective (which
    # sets up the communicator and can take a second) runs before the settle, so
    # the GPUs do not idle between their settle and the timed region.
    if world > 1:
        dist.barrier()
        sync()
    settle_n, ts = 0, time.perf_counter()
    while (time.perf_counter() - ts) * 1e3 < args.settle_ms and not args.dry_run:
        for _ in range(8):
            step()
        settle_n += 8
        sync()
    settle_ms = (time.perf_counter() - ts) * 1e3
    for _ in range(args.warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    if not args.dry_run:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if not args.dry_run:
        e0.record(stream)
    for _ in range(args.steps):
        step()
    if not args.dry_run:
        e1.record(stream)
    sync()
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    kern_ms = e0.elapsed_time(e1) / args.steps if not args.dry_run else 0.0  # launch stream
    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t[0])

    # every rank checks its whole timed batch (all N outputs) against the
    # reference over the same bytes, copied back from HBM
    cpus = host_cpus()
    verify, first_chunk = None, None
    if not args.no_verify and not args.dry_run:
        thr = max(1, usable_cpus(cpus) // max(1, local_world))
        verify, first_chunk = verify_timed_batch(
            b, base, out, thr, keep_first=(rank == 0 and world == 1 and not args.no_cpu_baseline))
        if not verify["ok"]:
            log(f"bench.py rank {rank}: {verify['mismatches']} of {b.n} checksums differ from the reference")

    # per-rank report: bytes, kernel time, verification
    mine = {"bytes": b.algo_bytes, "descriptors": b.n, "kernel_ms": kern_ms,
            "verified": None if verify is None else verify["ok"],
            "mismatches": None if verify is None else verify["mismatches"]}
    per_rank = [mine]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    total_bytes = sum(r["bytes"] for r in per_rank)
    value = total_bytes * args.steps / wall_max / 1e9 if wall_max > 0 else 0.0
    achieved = b.algo_bytes / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else 0.0  # rank 0's kernel
    achieved_c = (b.algo_bytes + 2 * b.n) / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else 0.0
    rank_ach = [r["bytes"] / (r["kernel_ms"] / 1e3) / 1e9 if r["kernel_ms"] > 0 else 0.0 for r in per_rank]
    for r, info, a in zip(per_rank, ranks, rank_ach):
        info.update({"kernel_ms": round(r["kernel_ms"], 5), "kernel_GBps": round(a, 2),
                     "descriptors": r["descriptors"], "verified": r["verified"]})
    verified = None
    if all(r["verified"] is not None for r in per_rank):
        verified = all(r["verified"] for r in per_rank)

    kernel_label = f"{args.kernel}-u{args.unroll}-w{args.waves_per_cu}"
    chosen = args.kernel
    launches = 1
    if not args.dry_run:
        if kernel == 0:
            chosen = lvlip.auto_kernel_name(len_hint, b.n)
        # a step is one batch_dev call; long k_window batches go out as several
        # launches (lvlip_batch_launches), and rocprof averages per launch
        launches = max(1, lvlip.batch_launches(b.n, kernel, args.unroll, args.waves_per_cu, len_hint))

    diag = {"settle": {"launches": settle_n, "ms": round(settle_ms, 1)}}
    if verify is not None:
        diag["verify"] = verify
    if scatter_diag is not None:
        diag["scatter"] = scatter_diag
    if rank == 0 and not args.dry_run:
        if args.sweep:
            diag["sweep"] = sweep(lvlip, torch, base, descs, out, b, stream)
        if base.numel() < (1 << 34):
            diag["read_probe_GBps"] = read_probe(lvlip, torch, base, stream)
        if args.frames:
            diag["frames_dev"] = frames_dev(lvlip, torch, dev)
        if (args.frames and not args.no_crossover) or args.crossover:
            diag["crossover"] = crossover(lvlip, dev)
        if args.e2e:
            diag["e2e_host_GBps"] = e2e(lvlip, b, base)
            diag["link_probe"] = link_probe(torch, dev, b.nbytes)
            diag["latency_us"] = latency(lvlip, torch, dev)

    cpu = None
    if rank == 0 and world == 1 and first_chunk is not None:
        cpu = cpu_baseline(b, first_chunk, cpus)

    if rank == 0:
        tr = traffic_from_profiles(args.workload, kernel_label, KERNEL_FN.get(chosen, ""))
        rec = {
            "metric": METRIC, "value": None if args.dry_run else round(value, 2), "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": None if args.dry_run else round(wall_max * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "strong" if args.workload in STRONG else "weak",
            "vs_baseline": None, "dtype": "u16",
            "data": "synthetic (splitmix64 seed 0x1E7E1C5, 1% all-0x00 + 1% all-0xff packets), "
                    "device-resident",
            "config": {"workload": f"{args.workload}: {WORKLOAD_TEXT[args.workload]}",
                       "descriptors_per_gpu": b.n, "bytes_per_gpu": b.algo_bytes,
                       "kernel": kernel_label, "kernel_selected": chosen,
                       "len_hint": len_hint, "parallelism": f"shard{world} (no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "frac_aggregate": round(value / (world * HBM_PEAK_GBPS), 4),
                         "frac_min_rank": round(min(rank_ach) / HBM_PEAK_GBPS, 4),
                         "traffic": tr[0] if tr else None,
                         "traffic_source": tr[1] if tr else None,
                         "kernel_ms": round(kern_ms, 5),
                         "launches_per_step": launches,
                         "kernel_ms_per_launch": round(kern_ms / launches, 5),
                         "algo_bytes_per_launch": b.algo_bytes // launches,
                         # SURVEY.md §8(d)'s algorithmic bytes: the bytes summed
                         # plus the 2-B results written (achieved above counts
                         # the summed bytes only, 0.13 % less on tcp1500)
                         "contract_bytes_per_launch": (b.algo_bytes + 2 * b.n) // launches,
                         "achieved_contract": round(achieved_c, 2),
                         "frac_contract": round(achieved_c / HBM_PEAK_GBPS, 4)},
            "cpu_baseline": cpu,
            "verified_bit_exact": verified,
            "dist": {"world_size": dist.get_world_size() if world > 1 else 1,
                     "backend": backend if world > 1 else None, "launcher": launcher,
                     "shared_devices": len({(r["host"], r.get("pci")) for r in ranks}) < world,
                     "ranks": ranks},
            "diag": diag,
        }
        if args.dry_run:
            rec["dry_run"] = True
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if verified is False:
        raise SystemExit("bench.py: the timed batch's checksums differ from the reference")


def timed(torch, fn, stream, reps=20, warm=3):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def sweep(lvlip, torch, base, descs, out, b, stream):
    res = {}
    variants = [("window", 2 | (4 << 8), 16), ("window", 2 | (4 << 8), 12), ("window", 2 | (2 << 8), 8),
                ("window", 2 | (3 << 8), 8), ("wave", 2, 8), ("wave", 2, 12), ("wave", 3, 12),
                ("flat", 4, 0), ("flat", 8, 0), ("flat", 8 | (2 << 8), 0), ("wflat", 0, 0)]
    for rnd in range(2):  # interleaved rounds in one process
        for k, u, w in variants:
            def f():
                lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(),
                                stream.cuda_stream, lvlip.KERNEL_NAMES[k], u, w)
            ms = timed(torch, f, stream, reps=10)
            key = f"{k}-u{u:#x}-w{w}"
            res.setdefault(key, []).append(round(b.algo_bytes / ms / 1e6, 1))
    for k, v in res.items():
        log(f"sweep {k:18s} GB/s {v}")
    return res


def mixed_frames_hbm(lvlip, torch, dev):
    """The mixed config's 2M frames made valid IPv4/TCP/ICMP frames in HBM
    (Ethernet type, version/ihl, total length, TTL, protocol written into each
    frame's header): (uint8 CUDA tensor, FRAME_DESC_DTYPE descriptors, the
    payload descriptors)."""
    import workloads

    b = workloads.make("mixed")
    base, _, _ = workloads.to_device(b, dev)
    hdr = b.descs[0::2]
    pay = b.descs[1::2]
    n = hdr.size
    fstart = torch.from_numpy((hdr["offset"] - 14).astype(np.int64)).to(dev)
    iplen = torch.from_numpy((20 + pay["len"]).astype(np.int64)).to(dev)
    proto = torch.from_numpy(np.where(pay["start_sum"] != 0, 6, 1).astype(np.int64)).to(dev)

    def put(k, vals):
        base[fstart + k] = vals.to(torch.uint8) if torch.is_tensor(vals) else vals

    put(12, 0x08), put(13, 0x00), put(14, 0x45), put(15, 0)
    put(16, iplen >> 8), put(17, iplen & 0xFF), put(22, 64), put(23, proto)
    fd = np.zeros(n, dtype=lvlip.FRAME_DESC_DTYPE)
    fd["offset"] = hdr["offset"] - 14
    fd["len"] = 34 + pay["len"]
    return base, fd, pay


def frames_dev(lvlip, torch, dev):
    """Device-resident frame batches (diagnostic, include/lvlip_skb.h): the mixed
    config's 2M frames made valid IPv4/TCP/ICMP frames in HBM, then TX fill,
    RX verify (header) and RX verify with L4, each timed with HIP events on
    the launch stream.  GB/s counts the checksummed bytes of each call."""
    base, fd, pay = mixed_frames_hbm(lvlip, torch, dev)
    n = fd.size
    fdt = torch.from_numpy(fd.view(np.uint8).copy()).to(dev)
    stream = torch.cuda.current_stream(dev)
    l4_bytes = int(pay["len"].sum())
    res = {}
    for name, fn, nbytes in (
            ("tx_fill", lambda: lvlip.tx_checksum_dev(base, fdt, stream=stream), 20 * n + l4_bytes),
            # A/B (liblvlip_lab.so): the same shape (U 8, blocks) with plain
            # (temporal) field stores
            ("tx_fill_plain", lambda: lvlip.frames_variant_dev(0, 1 | 2 | 4, base, fdt, stream=stream),
             20 * n + l4_bytes),
            ("rx_header", lambda: lvlip.rx_verify_dev(base, fdt, 0, stream=stream), 20 * n),
            # A/B: the header call on k_flat2 with a frame source
            ("rx_header_flat", lambda: lvlip.frames_variant_dev(1, 0, base, fdt, stream=stream), 20 * n),
            ("rx_header_l4", lambda: lvlip.rx_verify_dev(base, fdt, lvlip.RX_VERIFY_L4, stream=stream),
             20 * n + l4_bytes)):
        ms = timed(torch, fn, stream, reps=10)
        res[name] = {"ms": round(ms, 4), "Mframes_per_s": round(n / ms / 1e3, 1),
                     "GBps": round(nbytes / ms / 1e6, 1)}
    v = lvlip.rx_verify_dev(base, fdt, 0, stream=stream)
    torch.cuda.synchronize(dev)
    res["rx_header_all_ok"] = bool((v == lvlip.RX_OK).all())
    res["echo_reply"] = echo_reply_timing(lvlip, torch, base, fd, fdt, pay, stream)
    # the same frames from host memory through the host API (PCIe-inclusive),
    # on a 512K-frame prefix
    nh = min(n, 1 << 19)
    end = int(fd["offset"][nh - 1]) + int(fd["len"][nh - 1])
    host = base[: (end + 15) // 16 * 16].cpu().numpy().copy()
    res["host"] = frames_host(lvlip, dev, host, fd[:nh], int(pay["len"][:nh].sum()))
    res["host"]["link_probe"] = link_probe(torch, dev, host.nbytes)
    log("device-resident frames", res)
    return res


def echo_reply_timing(lvlip, torch, base, fd, fdt, pay, stream, reps=7):
    """f4 on the mixed frames in HBM: every ICMP frame made an
    echo request (type 8, code 0; its checksum field is whatever the TX fill
    left, so flags 0's field is the RFC 1624 one, not verified), then
    lvlip_icmp_echo_reply_dev with flags 0 (one 64-B sector per frame) and
    with LVLIP_ECHO_FULL (the flat sweep over the requests' messages), HIP
    events around each launch alone; the request bytes are restored before
    every launch.  Everything the call needs is made before the first event,
    so the pair holds the ctypes call and the kernel only (round 5's form
    made the status tensor between the events and read ~20 % slower than
    the kernel trace).  GB/s counts the ICMP messages' bytes."""
    icmp = pay["start_sum"] == 0
    t_off = torch.from_numpy((fd["offset"][icmp] + 34).astype(np.int64)).to(base.device)
    msg_bytes = int(pay["len"][icmp].sum())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {"icmp_frames": int(icmp.sum()), "icmp_bytes": msg_bytes}
    lib = lvlip.lib()
    n = fd.size
    st = torch.empty(n, dtype=torch.uint8, device=base.device)
    args = (base.data_ptr(), fdt.data_ptr(), n)
    for name, flags in (("flags0", 0), ("full", lvlip.ECHO_FULL)):
        ms = []
        for _ in range(reps):
            base[t_off] = 8
            base[t_off + 1] = 0
            torch.cuda.synchronize()
            e0.record(stream)
            if flags == 0:
                rc = lib.lvlip_icmp_echo_reply_dev(*args, st.data_ptr(), stream.cuda_stream)
            else:
                rc = lib.lvlip_icmp_echo_reply_dev_ex(*args, flags, st.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            assert rc == lvlip.OK, rc
            ms.append(e0.elapsed_time(e1))
        med = sorted(ms)[len(ms) // 2]
        out[name] = {"ms": round(med, 4), "GBps": round(msg_bytes / med / 1e6, 1),
                     "replies": int((st.cpu() != 0).sum())}
    return out


def cpu_header_check(lvlip, host, fd, budget_s=0.3):
    """What ip_rcv's header check costs on one host core (src/ip_input.c:38:
    checksum(ih, ihl * 4, 0) per received frame), to set beside the RX batch's
    host-path cost per frame: the n frames' 20-B IPv4 headers (frame + 14) of
    the host slab, level-ip's own checksum() (oracle/_ref, -O0 as built) and
    the product's per-call drop-in, ns per header (the CPU-baseline leg)."""
    import pyoracle  # test infrastructure: a reported CPU baseline only

    d = np.zeros(fd.size, dtype=lvlip.DESC_DTYPE)
    d["offset"] = fd["offset"] + 14
    d["len"] = 20
    res = {"headers": int(fd.size)}
    kinds = [("dropin_ns", {"csum_fn": lvlip.lib().checksum})]
    if pyoracle.reflib() is not None:
        kinds.insert(0, ("reference_O0_ns", {"use_reference": True}))
    # over the whole slab every header is a cache miss; in the stack ip_rcv
    # sums a header tun_read has just written: the first 2 048 frames' headers
    # 64 times over in one pass (in cache) give that case
    for tag, dd in (("", d), ("_cached", np.tile(d[:2048], 64))):
        for name, kw in kinds:
            reps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < budget_s:
                pyoracle.batch(host, dd, threads=1, **kw)
                reps += 1
            res[name.replace("_ns", tag + "_ns")] = round((time.perf_counter() - t0) / reps / dd.size * 1e9, 2)
    # what the RX + L4 call does per frame, on one core with the drop-in: the
    # 20-B header and the TCP/ICMP segment after it (two checksums per frame)
    d2 = np.zeros(2 * fd.size, dtype=lvlip.DESC_DTYPE)
    d2["offset"][0::2] = fd["offset"] + 14
    d2["len"][0::2] = 20
    d2["offset"][1::2] = fd["offset"] + 34
    d2["len"][1::2] = np.maximum(fd["len"].astype(np.int64) - 34, 0)
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        pyoracle.batch(host, d2, threads=1, csum_fn=lvlip.lib().checksum)
        reps += 1
    res["dropin_header_l4_ns_per_frame"] = round((time.perf_counter() - t0) / reps / fd.size * 1e9, 2)
    return res


def frames_host(lvlip, dev, host, fd, l4_bytes):
    """The host frame calls (include/lvlip_skb.h lvlip_tx_checksum,
    lvlip_rx_verify) on n frames in host memory, PCIe included, wall time per
    call (1 warm-up, then the mean of 5), from each source the library knows
    (frames_host.cpp):
      slab       the frames in one pageable buffer, as laid out in HBM (the
                 gather path: every frame one memcpy into the pinned arena)
      scattered  every frame at the start of its own 1616-B slot (a malloc'd
                 alloc_skb(BUFLEN) buffer, src/skbuff.c:5-20), the slots in
                 random order over an n x 1616 B buffer (the gather path)
      dma        the slab registered LVLIP_REG_DMA (copy engine reads spans)
      dma_shuffled  the same registered slab, the frames in shuffled call
                 order over a slab far larger than the arena (not
                 dense in order, so gathered frame by frame instead of cut
                 into one-frame pieces each moving a whole span)
      zerocopy   the slab registered LVLIP_REG_ZEROCOPY (kernel reads in place)
      scattered_t8  scattered with 8 gather threads (LVLIP_GATHER_THREADS;
                 the default is min(hardware threads, 16), round 4's was 8)
      slab_spin, dma_spin  slab and dma with every piece waited for by
                 spinning (LVLIP_BLOCK_MIN=0; the default sleeps on pieces
                 from 4 MiB)
    GB/s counts the checksummed bytes (20 B header + L4 per frame) as the
    device lines do; frame_GBps counts the frames' bytes (what crosses PCIe);
    cpu_ns_per_frame is the process's CPU time (all threads) per frame, what
    the call costs the host beside the CPU's own checksum (cpu_header_check)."""
    import ctypes

    n = fd.size
    hb = 20 * n + l4_bytes
    frame_bytes = int(fd["len"].sum())
    stride = 1616
    rng = np.random.default_rng(7)
    slot = rng.permutation(n)
    scat = np.zeros(n * stride, np.uint8)
    for i in range(n):
        o, ln = int(fd["offset"][i]), int(fd["len"][i])
        scat[int(slot[i]) * stride:int(slot[i]) * stride + ln] = host[o:o + ln]

    def frames_arr(buf, offsets):
        fr = np.zeros(n, dtype=[("head", "<u8"), ("len", "<u4"), ("pad", "<u4")])
        assert fr.dtype.itemsize == ctypes.sizeof(lvlip.Frame)
        fr["head"] = buf.ctypes.data + offsets
        fr["len"] = fd["len"]
        return fr, ctypes.cast(fr.ctypes.data, ctypes.POINTER(lvlip.Frame))

    lib = lvlip.lib()
    verdict = np.zeros(n, np.uint8)
    out = {"frames": n, "frame_bytes": frame_bytes, "checksummed_bytes": hb}

    def run(ctx, arr, tag):
        calls = (("tx_fill", lambda: lib.lvlip_tx_checksum(ctx._h, arr, n)),
                 ("rx_header", lambda: lib.lvlip_rx_verify(ctx._h, arr, n, 0, verdict.ctypes.data)),
                 ("rx_header_l4", lambda: lib.lvlip_rx_verify(ctx._h, arr, n, lvlip.RX_VERIFY_L4,
                                                              verdict.ctypes.data)))
        r = {}
        for name, call in calls:
            assert call() == 0, (tag, name)
            if name == "rx_header":  # filled by tx_fill (L4: the lossy TCP seed may not verify)
                assert (verdict == lvlip.RX_OK).all(), (tag, name)
            t0, c0 = time.perf_counter(), time.process_time()
            for _ in range(5):
                assert call() == 0, (tag, name)
            ms = (time.perf_counter() - t0) / 5 * 1e3
            cpu_ms = (time.process_time() - c0) / 5 * 1e3
            nb = 20 * n if name == "rx_header" else hb
            r[name] = {"ms": round(ms, 3), "Mframes_per_s": round(n / ms / 1e3, 2),
                       "GBps": round(nb / ms / 1e6, 2),
                       # CPU time of the whole process (every thread: the
                       # caller's wait, the pool's gather and apply) per frame
                       "cpu_ns_per_frame": round(cpu_ms * 1e6 / n, 2)}
            if name != "rx_header":
                r[name]["frame_GBps"] = round(frame_bytes / ms / 1e6, 2)
        out[tag] = r
        log(f"host frames {tag:9s}", {k: v["GBps"] for k, v in r.items()})

    keep_slab = frames_arr(host, fd["offset"].astype(np.uint64))
    keep_scat = frames_arr(scat, slot.astype(np.uint64) * stride)
    shuf = rng.permutation(n)
    keep_shuf = frames_arr(host, fd["offset"].astype(np.uint64))
    keep_shuf[0][:] = keep_shuf[0][shuf]
    d = dev.index or 0
    with lvlip.Context(d, cpu_max=0) as ctx:  # the GPU path (crossover() times both sides)
        run(ctx, keep_slab[1], "slab")
        run(ctx, keep_scat[1], "scattered")
        for tag, flag, arr in (("dma", lvlip.REG_DMA, keep_slab[1]), ("zerocopy", lvlip.REG_ZEROCOPY, keep_slab[1]),
                               ("dma_shuffled", lvlip.REG_DMA, keep_shuf[1])):
            ctx.register(host, flag)
            try:
                s0 = ctx.stats()
                run(ctx, arr, tag)
                s1 = ctx.stats()
                out[tag]["h2d_bytes_per_call"] = (s1["h2d_bytes"] - s0["h2d_bytes"]) // max(1, s1["gpu_calls"] -
                                                                                          s0["gpu_calls"])
            finally:
                ctx.unregister(host)
    for env, tag, arr, flag in (("LVLIP_GATHER_THREADS=8", "scattered_t8", keep_scat[1], None),
                                ("LVLIP_BLOCK_MIN=0", "slab_spin", keep_slab[1], None),
                                ("LVLIP_BLOCK_MIN=0", "dma_spin", keep_slab[1], lvlip.REG_DMA)):
        k, v = env.split("=")
        os.environ[k] = v
        try:
            with lvlip.Context(d, cpu_max=0) as ctx:
                if flag is not None:
                    ctx.register(host, flag)
                try:
                    run(ctx, arr, tag)
                finally:
                    if flag is not None:
                        ctx.unregister(host)
        finally:
            del os.environ[k]
    out["cpu_header_check"] = cpu_header_check(lvlip, host, fd)
    # the frames the TX calls filled are what the HBM frames hold after
    # tx_fill (same bytes, same fill): spot-check the slab against the scatter
    for i in range(0, n, max(1, n // 997)):
        o, ln = int(fd["offset"][i]), int(fd["len"][i])
        assert np.array_equal(host[o:o + ln], scat[int(slot[i]) * stride:int(slot[i]) * stride + ln]), i
    return out


def mixed_frames_host(lvlip, n):
    """The mixed config's first n frames made valid IPv4/TCP/ICMP frames in
    host memory (the same header fields mixed_frames_hbm writes): (uint8
    array, FRAME_DESC_DTYPE descriptors)."""
    import workloads

    b = workloads.make("mixed", n=n)
    host = b.host_bytes()
    hdr, pay = b.descs[0::2], b.descs[1::2]
    fs = (hdr["offset"] - 14).astype(np.int64)
    iplen = (20 + pay["len"]).astype(np.int64)
    for k, v in ((12, 0x08), (13, 0x00), (14, 0x45), (15, 0), (16, iplen >> 8), (17, iplen & 0xFF),
                 (22, 64), (23, np.where(pay["start_sum"] != 0, 6, 1))):
        host[fs + k] = v
    fd = np.zeros(n, dtype=lvlip.FRAME_DESC_DTYPE)
    fd["offset"] = fs
    fd["len"] = 34 + pay["len"]
    return host, fd


CROSS_N = (1, 3, 8, 64, 512, 2048, 4096, 8192, 16384, 32768, 65536, 262144)
SKB_DTYPE = np.dtype([("next", "<u8"), ("prev", "<u8"), ("rt", "<u8"), ("dev", "<u8"), ("refcnt", "<i4"),
                      ("protocol", "<u2"), ("pad", "<u2"), ("len", "<u4"), ("dlen", "<u4"), ("seq", "<u4"),
                      ("end_seq", "<u4"), ("end", "<u8"), ("head", "<u8"), ("data", "<u8"),
                      ("payload", "<u8")])  # struct sk_buff on LP64 (include/skbuff.h:9-23)
assert SKB_DTYPE.itemsize == 88 and SKB_DTYPE.fields["data"][1] == 72


def crossover(lvlip, dev, ns=CROSS_N, budget_s=0.12):
    """Where a context's host calls should leave the calling thread (VERDICT
    r05 Next #1; lvlip_csum_ctx_set_cpu_max).  For n = 1 .. 256K of the mixed
    config's frames, each host call is timed on both sides of the threshold in
    the same context: "gpu" (cpu_max 0: the device pipeline) and "cpu"
    (cpu_max 2^32-1: the library's CPU code on the calling thread, one core,
    the drop-in checksum() per field).  Per call: wall time (us, the mean over
    >= 3 calls after 2 warm-ups, including ~1 us of ctypes) and the process's
    CPU time (us, every thread: the caller's wait and the pool's gather on the
    GPU side).  Calls:
      tx, rx_hdr, rx_l4   lvlip_tx_checksum, lvlip_rx_verify (flags 0, L4)
      pkt_iov             lvlip_csum_batch_host over the frames' IPv4 headers
                          and L4 segments (2n packets, what INTEGRATION §2a's
                          per-field batch sends)
      tx_skb, rx_skb      the _skb_list forms over sk_buff_heads of n skbs
    Sources:
      slab        the frames packed in one pageable buffer, in order
      scattered   each frame at the start of its own alloc_skb(BUFLEN) slot
                  (1616 B), the slots in shuffled order: netdev_rx_loop's /
                  ip_output's skbs (src/netdev.c:86-101, src/skbuff.c:5-20)
      registered  the slab registered LVLIP_REG_DMA (f3)
    crossover[call/source] = the smallest n measured from which the GPU side's
    wall time stays below the CPU side's (null: never up to 256K)."""
    import ctypes

    n_max = max(ns)
    host, fd = mixed_frames_host(lvlip, n_max)
    lib = lvlip.lib()
    d = dev.index or 0
    stride = 1616
    rng = np.random.default_rng(9)
    slot = rng.permutation(n_max)
    scat = np.zeros(n_max * stride + 64, np.uint8)
    for i in range(n_max):
        o, ln = int(fd["offset"][i]), int(fd["len"][i])
        scat[int(slot[i]) * stride:int(slot[i]) * stride + ln] = host[o:o + ln]
    fr_dtype = np.dtype([("head", "<u8"), ("len", "<u4"), ("pad", "<u4")])
    frames = {}
    for tag, buf, offs in (("slab", host, fd["offset"].astype(np.uint64)),
                           ("scattered", scat, slot.astype(np.uint64) * np.uint64(stride))):
        fr = np.zeros(n_max, dtype=fr_dtype)
        fr["head"] = np.uint64(buf.ctypes.data) + offs
        fr["len"] = fd["len"]
        frames[tag] = fr
    frames["registered"] = frames["slab"]
    # iov over the headers and L4 segments (2 per frame, frame order)
    iovs = {}
    for tag, fr in frames.items():
        iov = np.zeros(2 * n_max, dtype=[("ptr", "<u8"), ("len", "<i4"), ("start_sum", "<u4")])
        iov["ptr"][0::2] = fr["head"] + np.uint64(14)
        iov["len"][0::2] = 20
        iov["ptr"][1::2] = fr["head"] + np.uint64(34)
        iov["len"][1::2] = fr["len"].astype(np.int64) - 34
        iovs[tag] = iov
    # skb queues over the scattered slots: RX as netdev_rx_loop leaves them
    # (data at the frame, end = data + BUFLEN), TX as ip_output leaves them
    # (data at the IPv4 header, len = the IP packet, 14 B reserved in front)
    skbs = {}
    for kind in ("rx", "tx"):
        s = np.zeros(n_max, dtype=SKB_DTYPE)
        a0 = s.ctypes.data
        s["next"] = np.uint64(a0) + np.arange(1, n_max + 1, dtype=np.uint64) * np.uint64(88)
        s["prev"] = np.uint64(a0) + (np.arange(n_max, dtype=np.uint64) - np.uint64(1)) * np.uint64(88)
        fr = frames["scattered"]
        if kind == "rx":
            s["data"] = s["head"] = fr["head"]
            s["end"] = fr["head"] + np.uint64(1600)
        else:
            s["head"] = fr["head"]
            s["data"] = fr["head"] + np.uint64(14)
            s["len"] = fr["len"] - 14
            s["end"] = fr["head"] + np.uint64(stride)
        skbs[kind] = s
    qheads = {k: np.zeros(3, dtype=np.uint64) for k in skbs}  # struct sk_buff_head: next, prev, qlen
    verdict = np.zeros(n_max, np.uint8)
    outp = np.zeros(2 * n_max, np.uint16)
    fp = {k: ctypes.cast(v.ctypes.data, ctypes.POINTER(lvlip.Frame)) for k, v in frames.items()}
    ip = {k: ctypes.cast(v.ctypes.data, ctypes.POINTER(lvlip.Iov)) for k, v in iovs.items()}

    def queue(kind, n):
        """An sk_buff_head over the first n skbs of `kind` (list_add_tail order)."""
        s, qh = skbs[kind], qheads[kind]
        h = qh.ctypes.data
        s["prev"][0] = h
        s["next"][:n - 1] = np.uint64(s.ctypes.data) + np.arange(1, n, dtype=np.uint64) * np.uint64(88)
        s["next"][n - 1] = h
        qh[0], qh[1], qh[2] = s.ctypes.data, s.ctypes.data + 88 * (n - 1), n
        return h

    def timeit(call):
        for _ in range(2):
            r = call()
            assert r >= 0, r
        reps, t0, c0 = 0, time.perf_counter(), time.process_time()
        while reps < 3 or time.perf_counter() - t0 < budget_s:
            call()
            reps += 1
        return ((time.perf_counter() - t0) / reps * 1e6, (time.process_time() - c0) / reps * 1e6)

    rows = {}
    for tag in ("slab", "scattered", "registered"):
        with lvlip.Context(d) as ctx:
            if tag == "registered":
                ctx.register(host, lvlip.REG_DMA)
            try:
                h, vp, op = ctx._h, verdict.ctypes.data, outp.ctypes.data
                f_, i_ = fp[tag], ip[tag]
                # each entry: n -> the call over the first n frames (queues built outside the timing)
                calls = {
                    "tx": lambda n: (lambda: lib.lvlip_tx_checksum(h, f_, n)),
                    "rx_hdr": lambda n: (lambda: lib.lvlip_rx_verify(h, f_, n, 0, vp)),
                    "rx_l4": lambda n: (lambda: lib.lvlip_rx_verify(h, f_, n, lvlip.RX_VERIFY_L4, vp)),
                    "pkt_iov": lambda n: (lambda: lib.lvlip_csum_batch_host(h, i_, 2 * n, op)),
                }
                if tag == "scattered":
                    def tx_skb(n):
                        q = queue("tx", n)
                        return lambda: lib.lvlip_tx_checksum_skb_list(h, q)

                    def rx_skb(n):
                        q = queue("rx", n)
                        return lambda: lib.lvlip_rx_verify_skb_list(h, q, 0, vp, n_max)
                    calls["tx_skb"], calls["rx_skb"] = tx_skb, rx_skb
                for name, make_call in calls.items():
                    r = {"gpu_us": [], "cpu_us": [], "gpu_cpu_time_us": [], "cpu_cpu_time_us": []}
                    for n in ns:
                        call = make_call(n)
                        for side, cm in (("gpu", 0), ("cpu", 0xFFFFFFFF)):
                            ctx.set_cpu_max(cm)
                            w, c = timeit(call)
                            r[f"{side}_us"].append(round(w, 2))
                            r[f"{side}_cpu_time_us"].append(round(c, 2))
                    rows[f"{name}/{tag}"] = r
                    log(f"crossover {name}/{tag}: gpu {r['gpu_us']} cpu {r['cpu_us']}")
            finally:
                if tag == "registered":
                    ctx.unregister(host)
    cross = {}
    for k, r in rows.items():
        cross[k] = None
        for j in range(len(ns)):
            if all(g < c for g, c in zip(r["gpu_us"][j:], r["cpu_us"][j:])):
                cross[k] = ns[j]
                break
    return {"n": list(ns), "frames": "mixed config (64-1460 B payloads, avg ~800 B frames)",
            "rows": rows, "crossover": cross}


def read_probe(lvlip, torch, base, stream):
    """Achievable streaming-read rate over the same buffer (lab probe; diagnostic)."""
    try:
        lab = lvlip.lab()
    except lvlip.LvlipUnavailable:
        return None
    sink = torch.zeros(1, dtype=torch.int32, device=base.device)
    nb = base.numel() & ~1023
    cus = torch.cuda.get_device_properties(base.device).multi_processor_count
    best = {}
    for mode, u, nt, bpc in ((1, 4, 1, 4), (1, 8, 1, 2), (3, 4, 0, 4)):
        ms = timed(torch, lambda: lab.lvlip_lab_probe(base.data_ptr(), nb, sink.data_ptr(), mode, u,
                                                      nt, cus * bpc, stream.cuda_stream),
                   stream, reps=10)
        best[f"m{mode}u{u}nt{nt}b{bpc}"] = round(nb / ms / 1e6, 1)
    # the chip-wide window order (4 KiB chunks dealt round robin, XCD-major,
    # 8 waves/CU): the best plain read of the buffer measured
    if cus % 4 == 0:
        ms = timed(torch, lambda: lab.lvlip_lab_probe_chunk(base.data_ptr(), nb, sink.data_ptr(), 4, 4, 1,
                                                            cus * 2, stream.cuda_stream),
                   stream, reps=10)
        best["window_c4"] = round(nb / ms / 1e6, 1)
    log("read_probe GB/s", best)
    return best


def link_probe(torch, dev, nbytes):
    """The host->device link's own rate, the ceiling of every host-resident
    line (diagnostic): nbytes from pinned host memory to HBM as one copy, and
    as 32 MiB copies back to back on one stream (the host pipelines' piece
    size, csum_ctx.cpp kPieceMax), GB/s; each the best of 3."""
    nbytes = min(int(nbytes), 1 << 31) & ~15
    src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    src.fill_(1)
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    piece = 32 << 20

    def bulk():
        dst.copy_(src, non_blocking=True)

    def pieces():
        for o in range(0, nbytes, piece):
            dst[o:o + piece].copy_(src[o:o + piece], non_blocking=True)

    # the host pipelines' shape: the pieces alternate over two streams (the
    # context's two slots), each piece followed by a small copy (a piece's
    # descriptors, 16 B per 1500-B packet)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    small = piece * 16 // 1504 & ~15

    def two_streams(with_small=False):
        for k, o in enumerate(range(0, nbytes, piece)):
            with torch.cuda.stream(streams[k & 1]):
                dst[o:o + piece].copy_(src[o:o + piece], non_blocking=True)
                if with_small:
                    dst[o:o + small].copy_(src[o:o + small], non_blocking=True)
        for s in streams:
            s.synchronize()

    res = {}
    for name, fn in (("h2d_bulk", bulk), ("h2d_32MiB_pieces", pieces),
                     ("h2d_32MiB_pieces_2streams", two_streams),
                     ("h2d_32MiB_pieces_2streams_desc", lambda: two_streams(True))):
        fn()
        stream.synchronize()
        best = 0.0
        for _ in range(3):
            t0 = time.perf_counter()
            fn()
            stream.synchronize()
            best = max(best, nbytes / (time.perf_counter() - t0) / 1e9)
        res[name + "_GBps"] = round(best, 2)
    res["bytes"] = nbytes
    log("link probe", res)
    del src, dst
    return res


def latency(lvlip, torch, dev):
    """Small-batch latency (diagnostic): one call's wall time for n x 1500 B,
    device-resident (launch + kernel, synchronised) and host-resident (gather +
    H2D + kernel + D2H).  Where a CPU per-call loop wins is read off these."""
    import workloads

    res = {}
    for n in (64, 1024, 16384):
        b = workloads.make("tcp1500", n=n)
        base, descs, out = workloads.to_device(b, dev)
        stream = torch.cuda.current_stream(dev)

        def f():
            lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), stream.cuda_stream,
                            lvlip.KERNEL_AUTO, 0, 0, 1500)
            stream.synchronize()

        for _ in range(20):
            f()
        t0 = time.perf_counter()
        for _ in range(200):
            f()
        res[f"dev_n{n}_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 1)
        host = b.host_bytes()
        with lvlip.Context(dev.index or 0, arena_bytes=64 << 20, cpu_max=0) as ctx:
            for _ in range(20):
                ctx.batch_host_flat(host, b.descs)
            t0 = time.perf_counter()
            for _ in range(100):
                ctx.batch_host_flat(host, b.descs)
            res[f"host_n{n}_us"] = round((time.perf_counter() - t0) / 100 * 1e6, 1)
    log("latency us", res)
    return res


def e2e(lvlip, b, base):
    """Host-resident batch, PCIe-inclusive: pinned gather + H2D + kernel + D2H
    (one flat buffer, lvlip_csum_batch_host_flat); the f3 paths over the same
    buffer registered in place (copy engine straight from it; kernel reading it
    over PCIe); and the same packets as an iov array, one pointer each
    (lvlip_csum_batch_host: a gather per packet)."""
    import ctypes

    host = np.ascontiguousarray(base.cpu().numpy()[: b.nbytes])
    # the same packets as an iov array (lvlip_csum_batch_host: one pointer per
    # packet, as the reference's call sites hold skb payloads)
    iov = np.zeros(b.n, dtype=[("ptr", "<u8"), ("len", "<i4"), ("start_sum", "<u4")])
    assert iov.dtype.itemsize == ctypes.sizeof(lvlip.Iov)
    iov["ptr"] = host.ctypes.data + b.descs["offset"]
    iov["len"] = b.descs["len"]
    iov["start_sum"] = b.descs["start_sum"]
    iov_p = ctypes.cast(iov.ctypes.data, ctypes.POINTER(lvlip.Iov))
    out = np.empty(b.n, np.uint16)
    lib = lvlip.lib()
    res = {}
    for name, flags in (("flat", None), ("registered_dma", lvlip.REG_DMA),
                        ("registered_zerocopy", lvlip.REG_ZEROCOPY), ("iov", None)):
        with lvlip.Context(base.device.index or 0, arena_bytes=256 << 20, cpu_max=0) as ctx:
            if flags is not None:
                ctx.register(host, flags)
            if name == "iov":
                def call():
                    assert lib.lvlip_csum_batch_host(ctx._h, iov_p, b.n, out.ctypes.data) == 0
            else:
                def call():
                    ctx.batch_host_flat(host, b.descs)
            call()
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                call()
            dt = (time.perf_counter() - t0) / reps
        res[f"{name}_GBps"] = round(b.algo_bytes / dt / 1e9, 2)
    log("e2e host-resident GB/s", res)
    return res


if __name__ == "__main__":
    main()
