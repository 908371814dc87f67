"""Lab (diagnostic, not the product): the host-resident pipeline's timeline.
Runs lvlip_csum_batch_host_flat over the tcp1500 batch (1M x 1500 B) in host
memory, REPS times from each source (the pinned-arena gather, a LVLIP_REG_DMA
region), so that rocprofv3 --kernel-trace --memory-copy-trace shows where the
link idles between pieces; prints each call's wall GB/s.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o t -- \\
        python3 scripts/lab_e2e_trace.py [REPS]
    python3 scripts/lab_e2e_trace.py --summary DIR    # gaps between H2D copies
    python3 scripts/lab_e2e_trace.py --ab WORKLOAD REPS ROUNDS ENVS SOURCES
        # env sets of ENVS (order0, default, piece64, piece128) interleaved
"""
import csv
import glob
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "level-ip_amd")]


ENVS = {"order0": {"LVLIP_COPY_ORDER": "0"}, "default": {},
        "piece64": {"LVLIP_PIECE_MAX": str(64 << 20)}, "piece128": {"LVLIP_PIECE_MAX": str(128 << 20)}}


def run(reps, envs=("default",), rounds=1, workload="tcp1500", sources=("gather", "dma")):
    """Each source's calls (best of reps per round) under each env set of
    ENVS, rounds interleaved; every call's results equal the first's.
    Sources: gather (lvlip_csum_batch_host_flat from plain memory), dma (the
    same buffer registered LVLIP_REG_DMA), iov (lvlip_csum_batch_host, one
    pointer per packet).  Returns {"env src": [GB/s per round]}."""
    import ctypes

    import lvlip
    import workloads

    b = workloads.make(workload)
    host = np.ascontiguousarray(b.host_bytes())
    iov = np.zeros(b.n, dtype=[("ptr", "<u8"), ("len", "<i4"), ("start_sum", "<u4")])
    iov["ptr"] = host.ctypes.data + b.descs["offset"]
    iov["len"] = b.descs["len"]
    iov["start_sum"] = b.descs["start_sum"]
    iov_p = ctypes.cast(iov.ctypes.data, ctypes.POINTER(lvlip.Iov))
    out = np.empty(b.n, np.uint16)
    lib = lvlip.lib()
    want = None
    res = {}
    for _ in range(rounds):
        for name in envs:
            for k in ("LVLIP_COPY_ORDER", "LVLIP_PIECE_MAX"):
                os.environ.pop(k, None)
            os.environ.update(ENVS[name])
            for src in sources:
                with lvlip.Context(0, arena_bytes=256 << 20) as ctx:
                    if src == "dma":
                        ctx.register(host, lvlip.REG_DMA)
                    if src == "iov":
                        def call():
                            assert lib.lvlip_csum_batch_host(ctx._h, iov_p, b.n, out.ctypes.data) == 0
                            return out.copy()
                    else:
                        def call():
                            return ctx.batch_host_flat(host, b.descs)
                    got = call()
                    if want is None:
                        want = got
                    assert np.array_equal(got, want), (name, src)
                    best = 0.0
                    for _ in range(reps):
                        t0 = time.perf_counter()
                        call()
                        dt = time.perf_counter() - t0
                        best = max(best, b.algo_bytes / dt / 1e9)
                        print(f"{name} {src}: {b.algo_bytes / dt / 1e9:.2f} GB/s ({dt * 1e3:.2f} ms)", flush=True)
                    res.setdefault(f"{name} {src}", []).append(round(best, 2))
                time.sleep(0.05)  # a visible gap between the sources in the trace
    for k in ("LVLIP_COPY_ORDER", "LVLIP_PIECE_MAX"):
        os.environ.pop(k, None)
    return res


def summary(d):
    """Per call (H2D copies separated by > 2 ms of idle), the link's busy
    share (the union of the copies' intervals: rocprofv3's copy records carry
    no byte count, so the piece copies are the H2D records over 100 us) and
    the idle gaps between consecutive piece copies."""
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"]))
    rows.sort()
    h2d = [r for r in rows if r[2].endswith("HOST_TO_DEVICE") and r[1] - r[0] > 100_000]
    calls, cur = [], []
    for r in h2d:
        if cur and r[0] - max(x[1] for x in cur) > 2_000_000:
            calls.append(cur)
            cur = []
        cur.append(r)
    if cur:
        calls.append(cur)
    for c in calls:
        t0, t1 = c[0][0], max(r[1] for r in c)
        busy, end = 0, t0
        for s, e, _ in c:  # union of the copies' intervals
            if e > end:
                busy += e - max(s, end)
                end = e
        gaps, end = [], c[0][1]
        for s, e, _ in c[1:]:
            if s > end:
                gaps.append((s - end) / 1e3)
            end = max(end, e)
        conc = sum(1 for k in range(1, len(c)) if c[k][0] < c[k - 1][1])
        print(f"{len(c)} piece copies in {(t1 - t0) / 1e6:.2f} ms: link busy {busy / (t1 - t0) * 100:.1f} %, "
              f"copy median {np.median([(e - s) / 1e3 for s, e, _ in c]):.1f} us, {conc} overlapping the "
              f"previous, {len(gaps)} idle gaps (median {np.median(gaps) if gaps else 0:.1f} us, "
              f"total {sum(gaps) / 1e3:.2f} ms)")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    elif len(sys.argv) > 1 and sys.argv[1] == "--ab":
        # --ab WORKLOAD REPS ROUNDS ENV,ENV,... SRC,SRC,...
        a = sys.argv[2:] + [None] * 5
        r = run(int(a[1] or 3), envs=tuple((a[3] or "order0,default").split(",")), rounds=int(a[2] or 3),
                workload=a[0] or "tcp1500", sources=tuple((a[4] or "gather,dma").split(",")))
        print("AB", r)
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
