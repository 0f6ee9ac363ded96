"""End-to-end (PCIe-inclusive) time split of one batch: upload (device image
build + H2D), solve, download, free.  usage: python scripts/e2e_breakdown.py [config] [n]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from deppy_amd import _lib  # noqa: E402
from tests.gpu_common import lowered_config  # noqa: E402

config = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
lw = lowered_config(config, n, 1000)
ctx = _lib.Context(0, 1)
ctx.solve(lw.rec_off, lw.rec)  # warm
for rep in range(3):
    t = [time.perf_counter()]
    r = ctx.upload(lw.rec_off, lw.rec); t.append(time.perf_counter())
    r.run(); t.append(time.perf_counter())
    r.download(); t.append(time.perf_counter())
    r.free(); t.append(time.perf_counter())
    ms = [round((b - a) * 1e3, 2) for a, b in zip(t, t[1:])]
    print(json.dumps({"config": config, "n": n, "upload_ms": ms[0], "run_ms": ms[1], "download_ms": ms[2],
                      "free_ms": ms[3], "total_ms": round(sum(ms), 2),
                      "res_per_s": round(n / sum(ms) * 1e3, 1), "rec_MB": round(4 * int(lw.rec_off[-1]) / 1e6, 1)}))
