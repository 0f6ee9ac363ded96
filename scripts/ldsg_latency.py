"""Config 5's largest catalogs one at a time on the mid-size placements: the
all-LDS multi-wave group (M_LDSG, DP_OPT_FORCE_LDSG) against the HBM-read
4-wave group (M_SPLIT4, DP_OPT_FORCE_MID) -- each catalog's kernel alone
(resident in HBM, median of 5 launches) and host to host (dp_solve) -- and one
oracle thread.  Run on the GPU box; DEPPY_VARIANT_LIB selects a variant build.

usage: python scripts/ldsg_latency.py [catalogs] [pool]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402
from tests.gpu_common import lowered_config  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 20
pool = int(sys.argv[2]) if len(sys.argv) > 2 else 300
lw = lowered_config(5, pool, 1000)  # int32 records: each placement stages its own form
nvs = np.array([int(lw.record(p)[1]) for p in range(pool)])
pick = [int(p) for p in np.argsort(-nvs)[:m]]
out = {"catalogs": m, "nv": [int(nvs[p]) for p in pick]}
for name, flags in (("ldsg", _lib.OPT_FORCE_LDSG), ("split4", _lib.OPT_FORCE_MID)):
    ctx = _lib.Context(0, 1, flags=flags)
    h2h, kern, st = [], [], []
    for p in pick:
        one = np.ascontiguousarray(lw.record(p))
        off = np.array([0, len(one)], np.int64)
        g = ctx.solve(off, one)
        st.append(int(g["status"][0]))
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
    ctx.close()
    out[name] = {"h2h_ms_median": round(float(np.median(h2h)) * 1e3, 4),
                 "kernel_ms_median": round(float(np.median(kern)), 4),
                 "kernel_ms_p90": round(float(np.percentile(kern, 90)), 4),
                 "kernel_ms": [round(x, 3) for x in kern], "status": st}
    print(name, json.dumps({k: v for k, v in out[name].items() if k != "kernel_ms"}), flush=True)
from oracle import oracle  # noqa: E402  (CPU side only)
c = []
for p in pick:
    one = np.ascontiguousarray(lw.record(p))
    off = np.array([0, len(one)], np.int64)
    t0 = time.perf_counter()
    oracle.solve_batch(off, one, 0, 1)
    c.append(time.perf_counter() - t0)
out["cpu_1thread_ms_median"] = round(float(np.median(c)) * 1e3, 4)
out["cpu_1thread_ms_p90"] = round(float(np.percentile(c, 90)) * 1e3, 4)
print(json.dumps(out))
