"""Lab (diagnostic, not the product): two builds of the product library in one
process, on the host-resident batch calls (lvlip_csum_batch_host_flat from
plain memory, from a LVLIP_REG_DMA and a LVLIP_REG_ZEROCOPY region, and
lvlip_csum_batch_host over an iov array), rounds interleaved.  The second
build is a library built from an earlier commit and placed at
level-ip_amd/build/prev/liblvlip_csum.so (git-ignored; it travels to the GPU
box with the tree):

    git worktree add /tmp/prev <commit> && make -C /tmp/prev/level-ip_amd \\
        /tmp/prev/level-ip_amd/liblvlip_csum.so
    mkdir -p level-ip_amd/build/prev && cp /tmp/prev/level-ip_amd/liblvlip_csum.so level-ip_amd/build/prev/
    python scripts/lab_lib_ab.py OUT.json [WORKLOAD] [ROUNDS]
    python scripts/lab_lib_ab.py OUT.json frames [ROUNDS]   # the host frame calls
    python scripts/lab_lib_ab.py OUT.json latency [ROUNDS]  # small host batches (64 MiB arena)

LAB_ARENA sets the contexts' arena bytes (default 256 MiB, as bench.py --e2e);
LAB_FRAME_SRC the frame calls' sources (default slab,dma; also zerocopy, scattered);
LAB_SRC the packet batches' sources (default gather,dma,zerocopy,iov; also
iov_dma, iov_zc: the iov call over the buffer registered);
LAB_PREV_LIB=cur makes "prev" this tree's library too, and LAB_ENV_CUR /
LAB_ENV_PREV ("K=V,K=V") set knobs for each side's contexts: an env A/B of
one build in one process.

Both libraries are driven through their C ABI only (ctypes); every call's
outputs are compared with the first call's.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "level-ip_amd")]


def bind(path):
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.lvlip_csum_ctx_create.argtypes = [ctypes.POINTER(vp), i32, ctypes.c_size_t]
    lib.lvlip_csum_ctx_destroy.argtypes = [vp]
    lib.lvlip_csum_register.argtypes = [vp, vp, ctypes.c_size_t, u32]
    lib.lvlip_csum_unregister.argtypes = [vp, vp]
    lib.lvlip_csum_batch_host_flat.argtypes = [vp, vp, ctypes.c_size_t, vp, u32, vp]
    lib.lvlip_csum_batch_host.argtypes = [vp, vp, u32, vp]
    lib.lvlip_tx_checksum.argtypes = [vp, vp, u32]
    lib.lvlip_rx_verify.argtypes = [vp, vp, u32, u32, vp]
    return lib


def ctx_create(name, lib, arena):
    """lvlip_csum_ctx_create under the environment LAB_ENV_<NAME> ("K=V,K=V";
    the context reads its knobs when it is made)."""
    env = os.environ.get(f"LAB_ENV_{name.upper()}", "")
    kv = [e.split("=", 1) for e in env.split(",") if e]
    old = {k: os.environ.get(k) for k, _ in kv}
    os.environ.update(dict(kv))
    try:
        h = ctypes.c_void_p()
        assert lib.lvlip_csum_ctx_create(ctypes.byref(h), 0, arena) == 0
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return h


def frames_ab(path, libs, rounds, arena, reps=3):
    """The host frame calls (TX fill, RX + L4) on 512K of bench.py's mixed
    frames in host memory, from a plain slab and from the slab registered
    LVLIP_REG_DMA, per library."""
    import torch

    import bench
    import lvlip

    dev = torch.device("cuda", 0)
    base, fd, pay = bench.mixed_frames_hbm(lvlip, torch, dev)
    fdt = torch.from_numpy(fd.view(np.uint8).copy()).to(dev)
    lvlip.tx_checksum_dev(base, fdt)
    torch.cuda.synchronize()
    n = min(fd.size, 1 << 19)
    end = int(fd["offset"][n - 1]) + int(fd["len"][n - 1])
    host = base[: (end + 15) // 16 * 16].cpu().numpy().copy()
    del base, fdt
    fr = np.zeros(n, dtype=[("head", "<u8"), ("len", "<u4"), ("pad", "<u4")])
    fr["head"] = host.ctypes.data + fd["offset"][:n].astype(np.uint64)
    fr["len"] = fd["len"][:n]
    # the same frames scattered: each at the start of its own 1616-B slot, the
    # slots in random order (bench.py --frames' scattered source)
    stride = 1616
    slot = np.random.default_rng(7).permutation(n)
    scat = np.zeros(n * stride, np.uint8)
    for i in range(n):
        o, ln = int(fd["offset"][i]), int(fd["len"][i])
        scat[int(slot[i]) * stride:int(slot[i]) * stride + ln] = host[o:o + ln]
    frs = fr.copy()
    frs["head"] = scat.ctypes.data + slot.astype(np.uint64) * stride
    hb = 20 * n + int(pay["len"][:n].sum())
    verdict = np.zeros(n, np.uint8)
    want = host.copy()
    res = {"frames": n, "arena": arena, "GBps": {}}
    for _ in range(rounds):
        for name, lib in libs.items():
            for src in os.environ.get("LAB_FRAME_SRC", "slab,dma").split(","):
                h = ctx_create(name, lib, arena)
                if src in ("dma", "zerocopy"):
                    flag = lvlip.REG_DMA if src == "dma" else lvlip.REG_ZEROCOPY
                    assert lib.lvlip_csum_register(h, host.ctypes.data, host.size, flag) == 0
                arr = frs if src == "scattered" else fr
                for call, fn in (("tx", lambda: lib.lvlip_tx_checksum(h, arr.ctypes.data, n)),
                                 ("rx_l4", lambda: lib.lvlip_rx_verify(h, arr.ctypes.data, n, lvlip.RX_VERIFY_L4,
                                                                       verdict.ctypes.data))):
                    assert fn() == 0
                    best = 0.0
                    c0 = time.process_time()
                    for _ in range(reps):
                        t0 = time.perf_counter()
                        assert fn() == 0
                        best = max(best, hb / (time.perf_counter() - t0) / 1e9)
                    cpu_ns = (time.process_time() - c0) / reps / n * 1e9
                    key = f"{name} {src} {call}"
                    res["GBps"].setdefault(key, []).append(round(best, 2))
                    res.setdefault("cpu_ns_per_frame", {}).setdefault(key, []).append(round(cpu_ns, 1))
                    print(key, res["GBps"][key], res["cpu_ns_per_frame"][key], flush=True)
                assert np.array_equal(host, want), (name, src)  # the TX fill is idempotent
                lib.lvlip_csum_ctx_destroy(h)
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


def latency_ab(path, libs, rounds, arena):
    """Small host batches (n x 1500 B from plain memory, lvlip_csum_batch_host_flat):
    the mean wall time of 100 synchronised calls per library, as bench.py
    --e2e's diag.latency_us times them."""
    import lvlip
    import workloads

    res = {"arena": arena, "us": {}}
    bs = {n: workloads.make("tcp1500", n=n) for n in (64, 1024, 16384)}
    for _ in range(rounds):
        for name, lib in libs.items():
            h = ctx_create(name, lib, arena)
            for n, b in bs.items():
                host = np.ascontiguousarray(b.host_bytes())
                d = np.ascontiguousarray(b.descs, dtype=lvlip.DESC_DTYPE)
                out = np.empty(b.n, np.uint16)

                def call():
                    assert lib.lvlip_csum_batch_host_flat(h, host.ctypes.data, host.size, d.ctypes.data, b.n,
                                                          out.ctypes.data) == 0
                for _ in range(20):
                    call()
                t0 = time.perf_counter()
                for _ in range(100):
                    call()
                key = f"{name} n{n}"
                res["us"].setdefault(key, []).append(round((time.perf_counter() - t0) / 100 * 1e6, 1))
                print(key, res["us"][key], flush=True)
            lib.lvlip_csum_ctx_destroy(h)
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


def main(path, workload="tcp1500", rounds=3, reps=3):
    import lvlip
    import workloads

    prev = os.environ.get("LAB_PREV_LIB", os.path.join(ROOT, "level-ip_amd", "build", "prev", "liblvlip_csum.so"))
    libs = {"cur": bind(lvlip.LIB_PATH), "prev": bind(lvlip.LIB_PATH if prev == "cur" else prev)}
    arena = int(os.environ.get("LAB_ARENA", 256 << 20))
    if workload == "frames":
        return frames_ab(path, libs, rounds, arena)
    if workload == "latency":
        return latency_ab(path, libs, rounds, int(os.environ.get("LAB_ARENA", 64 << 20)))
    b = workloads.make(workload)
    host = np.ascontiguousarray(b.host_bytes())
    d = np.ascontiguousarray(b.descs, dtype=lvlip.DESC_DTYPE)
    iov = np.zeros(b.n, dtype=[("ptr", "<u8"), ("len", "<i4"), ("start_sum", "<u4")])
    iov["ptr"] = host.ctypes.data + d["offset"]
    iov["len"] = d["len"]
    iov["start_sum"] = d["start_sum"]
    out = np.empty(b.n, np.uint16)
    want = None
    res = {"workload": workload, "arena": arena, "GBps": {}}
    for _ in range(rounds):
        for name, lib in libs.items():
            for src in os.environ.get("LAB_SRC", "gather,dma,zerocopy,iov").split(","):
                h = ctx_create(name, lib, arena)
                if src in ("dma", "zerocopy", "iov_dma", "iov_zc"):
                    flag = lvlip.REG_DMA if src in ("dma", "iov_dma") else lvlip.REG_ZEROCOPY
                    assert lib.lvlip_csum_register(h, host.ctypes.data, host.size, flag) == 0
                if src.startswith("iov"):
                    def call():
                        return lib.lvlip_csum_batch_host(h, iov.ctypes.data, b.n, out.ctypes.data)
                else:
                    def call():
                        return lib.lvlip_csum_batch_host_flat(h, host.ctypes.data, host.size, d.ctypes.data, b.n,
                                                              out.ctypes.data)
                assert call() == 0
                if want is None:
                    want = out.copy()
                assert np.array_equal(out, want), (name, src)
                best = 0.0
                for _ in range(reps):
                    t0 = time.perf_counter()
                    assert call() == 0
                    best = max(best, b.algo_bytes / (time.perf_counter() - t0) / 1e9)
                assert np.array_equal(out, want), (name, src)
                lib.lvlip_csum_ctx_destroy(h)
                key = f"{name} {src}"
                res["GBps"].setdefault(key, []).append(round(best, 2))
                print(key, res["GBps"][key], flush=True)
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "tcp1500",
         int(sys.argv[3]) if len(sys.argv) > 3 else 3)
