"""Diagnostic (stamps build): how many LDS-table rounds overflow and are
redone on the HBM arrays in the forced multi-wave parity workloads, and
whether those problems stay bit-exact against the oracle."""
import ctypes
import json
import os
import sys

os.environ["DEPPY_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from deppy_amd import _lib  # noqa: E402
from oracle import oracle  # noqa: E402  (checker only)
from tests.gpu_common import compare_results, lowered_config  # noqa: E402

L = _lib.lib()
L.dp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _lib.c_i64p]
NS = 56
out = {}
for flags, name in ((_lib.OPT_FORCE_MID, "split4"), (_lib.OPT_FORCE_GROUP, "split"),
                    (_lib.OPT_FORCE_MID | _lib.OPT_TINY_TABLE, "split4_tiny")):
    for cfg, n, seed in ((2, 300, 41), (5, 120, 42), (3, 500, 43)):
        ctx = _lib.Context(0, 1, flags=flags)
        lw = lowered_config(cfg, n, seed)
        r = ctx.upload(lw.rec_off, lw.rec)
        r.run()
        g = r.download()
        st = np.zeros(NS * n, np.int64)
        L.dp_debug_stamps(ctx.h, r.h, st.ctypes.data_as(_lib.c_i64p))
        r.free()
        ctx.close()
        redo = st.reshape(n, NS)[:, 41]
        o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
        out["%s_c%d" % (name, cfg)] = {"problems_with_redo": int((redo > 0).sum()), "redo_rounds": int(redo.sum()),
                                       "bit_exact": compare_results(g, o, n) == []}
print(json.dumps(out))
