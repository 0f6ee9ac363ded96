"""Where a single catalog's host-to-host latency goes (config 2, 20 catalogs):
ctx.solve (the bench's latency leg) beside the kernel time of the same
catalog resident in HBM, per placement (one wavefront, 4-wave and 8-wave
workgroups), and the oracle on one thread.  Run on the GPU box."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402
from tests.gpu_common import lowered_config  # noqa: E402

config = int(sys.argv[1]) if len(sys.argv) > 1 else 2
N = 20
lw = lowered_config(config, N, 1000, packed=True)
lw32 = lowered_config(config, N, 1000)
out = {}
for name, flags, L in (("lds", 0, lw), ("lds_i32", 0, lw32), ("mid", _lib.OPT_FORCE_MID, lw32),
                       ("group", _lib.OPT_FORCE_GROUP, lw32)):
    ctx = _lib.Context(0, 1, flags=flags)
    h2h, kern = [], []
    for p in range(N):
        a, b = int(L.rec_off[p]), int(L.rec_off[p + 1])
        off = np.array([0, b - a], np.int64)
        one = np.ascontiguousarray(L.rec[a:b])
        ctx.solve(off, one)
        t0 = time.perf_counter()
        ctx.solve(off, one)
        h2h.append(time.perf_counter() - t0)
        r = ctx.upload(off, one)
        r.run()
        ks = []
        for _ in range(5):
            r.run()
            ks.append(ctx.last_kernel_ms())
        r.free()
        kern.append(float(np.median(ks)))
    out[name] = {"h2h_ms_median": round(float(np.median(h2h)) * 1e3, 4),
                 "kernel_ms_median": round(float(np.median(kern)), 4),
                 "kernel_ms_max": round(float(np.max(kern)), 4)}
    print(name, json.dumps(out[name]), flush=True)
    ctx.close()
from oracle import oracle  # noqa: E402  (checker / CPU side only)
c = []
for p in range(N):
    a, b = int(lw32.rec_off[p]), int(lw32.rec_off[p + 1])
    off = np.array([0, b - a], np.int64)
    one = np.ascontiguousarray(lw32.rec[a:b])
    t0 = time.perf_counter()
    oracle.solve_batch(off, one, 0, 1)
    c.append(time.perf_counter() - t0)
reps, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < 1.0:
    oracle.solve_batch(lw32.rec_off, lw32.rec, 0, 1)
    reps += 1
out["cpu_1thread"] = {"one_call_ms_median": round(float(np.median(c)) * 1e3, 4),
                      "per_catalog_in_batch_ms": round((time.perf_counter() - t0) / reps / N * 1e3, 4)}
print("cpu", json.dumps(out["cpu_1thread"]), flush=True)
