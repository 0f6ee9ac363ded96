"""Per-phase shader cycles per problem from the diagnostic stamps build
(DEPPY_STAMPS=1, libdeppy_hip_stamps.so): [init, base, search, epilogue, core]."""
import ctypes
import json
import os
import sys

os.environ["DEPPY_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from deppy_amd import _lib  # noqa: E402
from tests.gpu_common import lowered_config  # noqa: E402

L = _lib.lib()
L.dp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _lib.c_i64p]
config = int(sys.argv[1]) if len(sys.argv) > 1 else 2
ctx = _lib.Context(0, 1)
for n in (64, 10000):
    lw = lowered_config(config, n, 1000)
    r = ctx.upload(lw.rec_off, lw.rec)
    r.run()
    r.run()
    res = r.download()
    st = np.zeros(10 * n, np.int64)
    L.dp_debug_stamps(ctx.h, r.h, st.ctypes.data_as(_lib.c_i64p))
    r.free()
    st = st.reshape(n, 10)
    names = ["init", "base", "search", "epilogue", "core", "round_eval", "round_finish", "rounds", "rounds_1lit", "push_guess"]
    out = {"n": n, "kernel_ms": ctx.last_kernel_ms()}
    for cls, mask in [("all", np.ones(n, bool)), ("sat_A", (res["status"] == 1) & ((res["flags"] & 2) == 0)),
                      ("sat_B", (res["status"] == 1) & ((res["flags"] & 2) != 0)), ("unsat", res["status"] == -1)]:
        if mask.sum() == 0:
            continue
        out[cls] = {"count": int(mask.sum()),
                    **{nm: [int(np.mean(st[mask, i])), int(np.percentile(st[mask, i], 99))] for i, nm in enumerate(names)},
                    "total_mean": int(st[mask, :5].sum(1).mean()), "total_max": int(st[mask, :5].sum(1).max())}
    print(json.dumps(out), flush=True)
