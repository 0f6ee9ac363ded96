"""Host lowering throughput (dp_lower_into, storage reused): wire -> records."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402

out = {}
for cfg, n in ((2, 10000), (3, 100000), (5, 10000), (4, 32)):
    w = _lib.generate(cfg, n, 1000)
    wa = _lib.WireArrays(**{k: w[k] for k in ("prob_var_off", "var_id", "var_con_off", "con_kind", "con_n",
                                              "con_arg_off", "con_arg", "str_off")}, str_bytes=w["str_bytes"].tobytes())
    lw = _lib.Lowered(wa)
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        lw.relower(wa)
        reps += 1
    dt = (time.perf_counter() - t0) / reps
    out["config%d" % cfg] = {"res_per_s": round(n / dt, 1), "problems": n, "exact_path": lw.n_exact,
                             "threads": os.environ.get("DEPPY_HOST_THREADS", "auto")}
print(json.dumps(out))
