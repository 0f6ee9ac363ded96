"""Per-phase shader cycles per problem from the diagnostic stamps build
(DEPPY_STAMPS=1, libdeppy_hip_stamps.so): [init, base, search, epilogue, core],
five counters, and the wall-clock (100 MHz) start/end of every wave, to see
what the step's tail is made of."""
import ctypes
import json
import os
import sys

os.environ["DEPPY_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from deppy_amd import _lib  # noqa: E402
from tests.gpu_common import lowered_config  # noqa: E402

NS = 56
NAMES = ["init", "base", "search", "epilogue", "core", "round_total", "round_visit", "rounds",
         "rounds_1lit", "push_guess"]
EXTRA = {16: "search_solve", 17: "pop_guess", 18: "pushes", 19: "visit_1lit", 20: "visit_flat", 21: "flush_cards",
         22: "learned", 23: "n_watch_1lit", 24: "n_front_flat", 25: "n_learned_rows", 26: "n_cards",
         27: "init_stage", 28: "init_validate", 29: "init_build",
         32: "first_violated", 33: "analyze", 34: "n_first_violated", 35: "truncate", 36: "save_model",
         37: "push_pre", 38: "n_analyze", 39: "search_loop", 40: "loop_gap", 41: "lds_table_redo", 42: "n_flat_entries", 43: "mw_flat_ranges", 44: "mw_flat_wbuf", 45: "mw_flat_visits", 46: "lds_round_exchange", 47: "lds_round_commit", 48: "build_count", 49: "build_scan", 50: "build_fill"}
L = _lib.lib()
L.dp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _lib.c_i64p]
config = int(sys.argv[1]) if len(sys.argv) > 1 else 2
sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [64, 10000]
ctx = _lib.Context(0, 1)
for n in sizes:
    lw = lowered_config(config, n, 1000, packed=os.environ.get("DEPPY_PHASES_FORM") == "packed")
    r = ctx.upload(lw.rec_off, lw.rec)
    r.run()
    r.run()
    res = r.download()
    st = np.zeros(NS * n, np.int64)
    L.dp_debug_stamps(ctx.h, r.h, st.ctypes.data_as(_lib.c_i64p))
    r.free()
    st = st.reshape(n, NS)
    out = {"n": n, "kernel_ms": ctx.last_kernel_ms()}
    cyc = st[:, :5].sum(1)
    for cls, mask in [("all", np.ones(n, bool)), ("sat_A", (res["status"] == 1) & ((res["flags"] & 2) == 0)),
                      ("sat_B", (res["status"] == 1) & ((res["flags"] & 2) != 0)), ("unsat", res["status"] == -1)]:
        if mask.sum() == 0:
            continue
        out[cls] = {"count": int(mask.sum()),
                    **{nm: [int(np.mean(st[mask, i])), int(np.percentile(st[mask, i], 99))] for i, nm in enumerate(NAMES)},
                    **{nm: [int(np.mean(st[mask, i])), int(np.percentile(st[mask, i], 99))] for i, nm in EXTRA.items()},
                    "total_mean": int(cyc[mask].mean()), "total_max": int(cyc[mask].max())}
    # wall-clock timeline (us): when waves start / end relative to the first start
    w0 = st[:, 10].min()
    s_us = (st[:, 10] - w0) / 100.0
    e_us = (st[:, 11] - w0) / 100.0
    out["timeline_us"] = {"span": float(e_us.max()), "start_p50": float(np.median(s_us)),
                          "start_max": float(s_us.max()),
                          "end_p50": float(np.median(e_us)), "end_p90": float(np.percentile(e_us, 90)),
                          "end_p99": float(np.percentile(e_us, 99)), "end_max": float(e_us.max()),
                          "dur_mean": float((e_us - s_us).mean()), "dur_max": float((e_us - s_us).max())}
    top = np.argsort(-(e_us - s_us))[:15]
    out["slowest"] = [{"pid": int(p), "status": int(res["status"][p]), "flags": int(res["flags"][p]),
                       "steps": int(res["steps"][p]), "start_us": round(float(s_us[p]), 1),
                       "dur_us": round(float(e_us[p] - s_us[p]), 1),
                       **{nm: int(st[p, i]) for i, nm in enumerate(NAMES)}} for p in top]
    print(json.dumps(out), flush=True)
