"""Config 4 (OLM-scale catalogs, V~55k) on the GPU: time and bit-exact check.

usage: python scripts/config4.py [n_problems] [reps]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402
from oracle import oracle  # noqa: E402  (checker only)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
w = _lib.generate(4, n, 4000)
lw = _lib.Lowered(_lib.WireArrays(**{k: w[k] for k in (
    "prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off", "con_arg",
    "str_off")}, str_bytes=w["str_bytes"].tobytes()))
ctx = _lib.Context(0, 1)
r = ctx.upload(lw.rec_off, lw.rec)
r.run()
ts, kms = [], []
for _ in range(reps):
    t0 = time.perf_counter()
    r.run()
    ts.append(time.perf_counter() - t0)
    kms.append(ctx.last_kernel_ms())
g = r.download()
t0 = time.perf_counter()
o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
tcpu = time.perf_counter() - t0
ok = {k: bool(np.array_equal(g[k], o[k])) for k in ("status", "flags", "steps", "core_len", "installed")}
print(json.dumps({"n": n, "wall_ms": [round(t * 1e3, 3) for t in ts], "kernel_ms": [round(x, 3) for x in kms],
                  "res_per_s": round(n / min(ts), 2), "oracle_s_16thr": round(tcpu, 3), "parity": ok,
                  "status": np.unique(g["status"], return_counts=True)[1].tolist(),
                  "steps": g["steps"].tolist()[:16], "flags": g["flags"].tolist()[:16]}), flush=True)
