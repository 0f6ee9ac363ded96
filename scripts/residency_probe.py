"""Config 2 kernel-only rate on subsets of the batch by catalog size: does
dropping the few catalogs whose LDS footprint sets the launch's residency
(the launch requests its largest footprint) speed up the rest?"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402
from tests.gpu_common import lowered_config  # noqa: E402

lw = lowered_config(2, 12000, 1000, packed=True)
nv = lw.rec[lw.rec_off[:-1] + 1]
ctx = _lib.Context(0, 1)
out = {}
for name, keep in (("all", nv >= 0), ("nv<=264", nv <= 264), ("nv<=200", nv <= 200)):
    idx = np.flatnonzero(keep)[:10000] if name != "nv<=200" else np.flatnonzero(keep)
    parts = [lw.record(int(p)) for p in idx]
    off = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.int64)
    rec = np.concatenate(parts).astype(np.int32)
    n = len(idx)
    slots = [ctx.upload(off, rec) for _ in range(4)]
    for s in slots:
        s.run()
    t0 = time.perf_counter()
    K = 16
    for i in range(K):
        s = slots[i % 4]
        if i >= 4:
            s.wait()
        s.launch()
    for s in slots:
        s.wait()
    dt = time.perf_counter() - t0
    slots[0].run()
    ms = ctx.last_kernel_ms()
    for s in slots:
        s.free()
    out[name] = {"catalogs": n, "res_per_s": round(n * K / dt, 1), "serial_launch_ms": round(ms, 4),
                 "mean_nv": round(float(nv[idx].mean()), 1)}
print(json.dumps(out))
