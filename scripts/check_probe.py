"""Diagnostic build only (libdeppy_hip_stamps.so): run a batch through one
placement and report the kernel's failed index checks (DP_CHK) per problem.

usage: python scripts/check_probe.py <config> <n> <flags>
"""
import ctypes
import os
import sys

os.environ["DEPPY_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from deppy_amd import _lib  # noqa: E402
from oracle import oracle  # noqa: E402  (checker only)
from tests.gpu_common import compare_results, lowered_config  # noqa: E402

NS = 32
config, n, flags = (int(x) for x in sys.argv[1:4])
L = _lib.lib()
L.dp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _lib.c_i64p]
lw = lowered_config(config, n, 77)
ctx = _lib.Context(0, 1, flags=flags)
r = ctx.upload(lw.rec_off, lw.rec)
r.run()
g = r.download()
st = np.zeros(NS * n, np.int64)
L.dp_debug_stamps(ctx.h, r.h, st.ctypes.data_as(_lib.c_i64p))
st = st.reshape(n, NS)
bad_chk = np.nonzero(st[:, 15])[0]
print("problems with failed checks:", len(bad_chk), flush=True)
for p in bad_chk[:20]:
    print("  pid", p, "code", st[p, 12], "value", st[p, 13], "bound", st[p, 14], "count", st[p, 15],
          "status", g["status"][p], "nv", lw.record(p)[1], flush=True)
o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
bad = compare_results(g, o, n)
print("mismatches", len(bad), bad[:5], flush=True)
