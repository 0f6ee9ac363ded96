"""Config 2 kernel-only rate vs batches in flight (device-resident slots,
each its own stream): how much do more concurrent launches hide the tail?"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402
from tests.gpu_common import lowered_config  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = 10000
lw = lowered_config(cfg, n, 1000, packed=True)
ctx = _lib.Context(0, 1)
out = {}
for depth in (2, 4, 8, 12):
    slots = [ctx.upload(lw.rec_off, lw.rec) for _ in range(depth)]
    for s in slots:
        s.run()
    K = 48
    t0 = time.perf_counter()
    for i in range(K):
        s = slots[i % depth]
        if i >= depth:
            s.wait()
        s.launch()
    for s in slots:
        s.wait()
    dt = time.perf_counter() - t0
    for s in slots:
        s.free()
    out[depth] = round(n * K / dt, 1)
print(json.dumps({"config": cfg, "kernel_only_res_per_s_by_depth": out}))
