"""Times a context's first calls (round 6 diagnosis): a 64-frame warm call
(one direct piece), then a 15 654-frame TX call (two pieces, the second
through the copy engine) three times.  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "level-ip_amd"))
import lvlip  # noqa: E402
import workloads  # noqa: E402

t0 = time.perf_counter()
ctx = lvlip.Context(0, cpu_max=0)
res = {"create_ms": (time.perf_counter() - t0) * 1e3}
small = workloads.frames(64, seed=1)
big = workloads.frames(15654, seed=2)
for tag, fr in (("warm64", small), ("big1", big), ("big2", big), ("big3", big)):
    t = time.perf_counter()
    ctx.tx_checksum(fr)
    res[tag + "_ms"] = (time.perf_counter() - t) * 1e3
ctx.close()
print(json.dumps(res))
