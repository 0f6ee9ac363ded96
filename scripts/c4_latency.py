"""Config 4 (OLM-scale catalogs) one at a time: for each of the bench's first
catalogs, host to host through dp_solve (as bench.py's latency leg: the
record copied out of the batch, so it is staged), the kernel alone (resident,
second launch), and one oracle thread.  One JSON line per catalog, then the
medians.  Run under DEPPY_VARIANT_LIB to measure another build on the same
catalogs (scripts/mkvariant.sh).

usage: python scripts/c4_latency.py [catalogs] [seed]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib, shard  # noqa: E402
from oracle import oracle  # noqa: E402  (the CPU side and the check)

m = int(sys.argv[1]) if len(sys.argv) > 1 else 20
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
first = shard.shard_seed(seed, 0, 256)  # bench.py --config 4's catalogs
w = _lib.generate(4, m, first)
wa = _lib.WireArrays(**{k: w[k] for k in ("prob_var_off", "var_id", "var_con_off", "con_kind", "con_n",
                                          "con_arg_off", "con_arg", "str_off")}, str_bytes=w["str_bytes"].tobytes())
lw = _lib.Lowered(wa)  # int32 records (what config 4 lowers to in any form)
ctx = _lib.Context(0, 1, flags=int(os.environ.get("DEPPY_C4_FLAGS", "0")))  # (placement A/B: 4 = 4-wave groups)
rows = []
for p in range(m):
    one = np.ascontiguousarray(lw.record(p))
    off = np.array([0, len(one)], np.int64)
    ctx.solve(off, one)
    t0 = time.perf_counter()
    g = ctx.solve(off, one)
    h2h = time.perf_counter() - t0
    r = ctx.upload(off, one)
    r.run()
    r.run()
    kms = ctx.last_kernel_ms()
    r.free()
    t0 = time.perf_counter()
    o = oracle.solve_batch(off, one, 0, 1)
    cpu = time.perf_counter() - t0
    ok = all(np.array_equal(g[k], o[k]) for k in ("status", "flags", "steps", "installed"))
    row = {"catalog": p, "h2h_ms": round(h2h * 1e3, 3), "kernel_ms": round(kms, 3), "cpu_1thread_ms": round(cpu * 1e3, 3),
           "status": int(g["status"][0]), "class_b": bool(g["flags"][0] & 2), "steps": int(g["steps"][0]), "exact": ok}
    rows.append(row)
    print(json.dumps(row), flush=True)
med = {k: round(float(np.median([r[k] for r in rows])), 3) for k in ("h2h_ms", "kernel_ms", "cpu_1thread_ms")}
med.update({"catalogs": m, "lib": os.environ.get("DEPPY_VARIANT_LIB", "libdeppy_hip.so"),
            "all_exact": all(r["exact"] for r in rows)})
print(json.dumps({"median": med}), flush=True)
