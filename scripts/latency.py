"""Kernel time vs batch size (config 2): separates single-wave latency from
throughput under load.  Run on the GPU box."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402
from tests.gpu_common import lowered_config  # noqa: E402

config = int(sys.argv[1]) if len(sys.argv) > 1 else 2
lw = lowered_config(config, 40000, 1000)
ctx = _lib.Context(0, 1)
out = []
for n in [1, 8, 64, 256, 1024, 2304, 4608, 10000, 20000, 40000]:
    r = ctx.upload(lw.rec_off[:n + 1], lw.rec[:int(lw.rec_off[n])])
    for _ in range(3):
        r.run()
    ms = []
    for _ in range(10):
        r.run()
        ms.append(ctx.last_kernel_ms())
    r.free()
    out.append({"n": n, "kernel_ms": float(np.median(ms)), "us_per_problem": 1e3 * float(np.median(ms)) / n})
    print(json.dumps(out[-1]), flush=True)
