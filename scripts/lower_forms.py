"""Host lowering throughput per record form (dp_lower_into, storage reused):
int32, 16-bit (NARROW), packed (NARROW | PACKED: P16D / P16)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402

out = {}
for cfg, n in ((2, 10000), (3, 100000)):
    w = _lib.generate(cfg, n, 1000)
    wa = _lib.WireArrays(**{k: w[k] for k in ("prob_var_off", "var_id", "var_con_off", "con_kind", "con_n",
                                              "con_arg_off", "con_arg", "str_off")}, str_bytes=w["str_bytes"].tobytes())
    for name, kw in (("int32", {}), ("narrow", {"narrow": True}), ("packed", {"narrow": True, "packed": True})):
        lw = _lib.Lowered(wa, **kw)
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 2.0:
            lw.relower(wa)
            reps += 1
        dt = (time.perf_counter() - t0) / reps
        out["config%d_%s" % (cfg, name)] = round(n / dt, 1)
print(json.dumps(out))
