"""Where the SolveBatch path's time goes (config 2, 10k catalogs): the whole
batch lowered then solved (sat.solve_wire as in round 4), the pipelined
sub-batches (sat.SUB_BATCH), and each piece timed alone.  Run on the GPU box."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib, sat  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
w = _lib.generate(cfg, n, 1000)
wa = _lib.WireArrays(**{k: w[k] for k in ("prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off",
                                          "con_arg", "str_off")}, str_bytes=w["str_bytes"].tobytes())
ctx = _lib.Context(0, 1)


def t(f, reps=5):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e3, 3)


lw = _lib.Lowered(wa, **sat.LOWER_FLAGS)
print("lower whole ms", t(lambda: lw.relower(wa)))
print("solve whole ms (ctx.solve)", t(lambda: ctx.solve(lw.rec_off, lw.rec)))
print("submit+wait whole ms", t(lambda: ctx.submit(lw.rec_off, lw.rec).wait()))
for sb in (2048, 4096, 8192):
    subs = [wa.slice(a, min(n, a + sb)) for a in range(0, n, sb)]
    lws = [_lib.Lowered(subs[0], **sat.LOWER_FLAGS), _lib.Lowered(subs[0], **sat.LOWER_FLAGS)]
    print("sub %d: lower each ms" % sb, [t(lambda s=s: lws[0].relower(s), 3) for s in subs])
    lws[0].relower(subs[0])
    print("sub %d: submit+wait one ms" % sb, t(lambda: ctx.submit(lws[0].rec_off, lws[0].rec).wait(), 3))
    sat.SUB_BATCH = sb
    sat._lowering.pipe = None
    print("sub %d: solve_wire pipelined ms" % sb, t(lambda: sat.solve_wire(wa, ctx)))
sat.SUB_BATCH = 1 << 30
print("solve_wire whole ms", t(lambda: sat.solve_wire(wa, ctx)))
