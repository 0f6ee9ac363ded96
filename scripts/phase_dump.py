"""Per-problem phase stamps (diagnostic build) saved as npz for offline
analysis: record size, variables, status, flags, total cycles, wall start/end.
usage: DEPPY_STAMPS=1 python scripts/phase_dump.py <config> <n> <out.npz>"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from deppy_amd import _lib  # noqa: E402
from tests.gpu_common import lowered_config  # noqa: E402

NS = 32
L = _lib.lib()
L.dp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _lib.c_i64p]
config, n, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
ctx = _lib.Context(0, 1)
lw = lowered_config(config, n, 1000)
r = ctx.upload(lw.rec_off, lw.rec)
r.run()
r.run()
res = r.download()
st = np.zeros(NS * n, np.int64)
L.dp_debug_stamps(ctx.h, r.h, st.ctypes.data_as(_lib.c_i64p))
r.free()
off = np.asarray(lw.rec_off)
rec = np.asarray(lw.rec)
np.savez(out, stamps=st.reshape(n, NS), words=rec[off[:-1] + 10], nv=rec[off[:-1] + 1],
         status=res["status"], flags=res["flags"], steps=res["steps"], kernel_ms=ctx.last_kernel_ms())
print("saved", out, ctx.last_kernel_ms())
