#!/usr/bin/env python3
"""Prints gfx950's buffer_load_dwordx4 out-of-range behaviour (lab_probe.hip k_oob)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import torch  # noqa: E402

import lvlip  # noqa: E402

lab = lvlip.lab()
lab.lvlip_lab_oob.restype = ctypes.c_int
lab.lvlip_lab_oob.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
buf = torch.arange(1, 65, dtype=torch.uint8, device="cuda")  # bytes 0x01..0x40
out = torch.zeros(72 * 4, dtype=torch.int64, device="cuda").view(torch.int32)[: 72 * 4]
out = torch.zeros(72 * 4, dtype=torch.int32, device="cuda")
assert lab.lvlip_lab_oob(buf.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
torch.cuda.synchronize()
o = out.cpu().numpy().astype("uint32").reshape(24, 3, 4)
for nr in range(24):
    print(f"nr={nr:2d}", "  ".join(f"b{b}:" + " ".join(f"{o[nr, b, k]:08x}" for k in range(4))
                                   for b in range(3)))
