"""Loaders for tests/golden/* (plain data: JSON and allow_pickle=False npz)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def kats():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        k = json.load(f)
    out = []
    for c in k["checksum"]:
        if c["data_hex"] is not None:
            data = bytes.fromhex(c["data_hex"])
        else:
            g = c["data_gen"]
            if g["kind"] == "fill":
                data = bytes([g["byte"]]) * g["n"]
            else:
                data = bytes(((g["mul"] * i + g["add"]) & 0xFF) for i in range(g["n"]))
        out.append((c["name"], data, c["count"], c["start_sum"], c["expected"]))
    return out, k["tcp_udp_checksum"]


def vectors():
    return _npz("vectors.npz")


def tcp():
    return _npz("tcp.npz")


def iphdr():
    return _npz("iphdr.npz")


def echo():
    with open(os.path.join(GOLDEN, "echo.json")) as f:
        return json.load(f)


def tcp_frames():
    """TCP frames the reference stack transmitted (tests/ref_stack_child.py)."""
    with open(os.path.join(GOLDEN, "tcp_frames.json")) as f:
        d = json.load(f)
    return [bytes.fromhex(h) for h in d["frames"]]
