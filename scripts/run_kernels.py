#!/usr/bin/env python3
"""Runs chosen kernels on one resident workload (for rocprofv3 passes):
  RK_WORKLOAD=tcp1500 RK_KERNELS=window,wave RK_REPS=10 python3 scripts/run_kernels.py
An entry may carry a launch shape, kernel:unroll:waves_per_cu (bench.py's
names; unroll in any base, e.g. window:0x802:12)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402

b = workloads.make(os.environ.get("RK_WORKLOAD", "tcp1500"))
base, descs, out = workloads.to_device(b)
hint = b.algo_bytes // b.n
for _ in range(int(os.environ.get("RK_REPS", "10"))):
    for spec in os.environ.get("RK_KERNELS", "window,wave").split(","):
        f = spec.split(":")
        lvlip.batch_torch(base, descs, out, kernel=lvlip.KERNEL_NAMES[f[0]],
                          unroll=int(f[1], 0) if len(f) > 1 else 0,
                          waves_per_cu=int(f[2]) if len(f) > 2 else 0, len_hint=hint)
torch.cuda.synchronize()
print("ok")
