"""Device lowering alone (dp_lower_device), per call: config C, n catalogs,
k calls into one reused result; prints the median call time and the host
lowering's (dp_lower_into) for the same batch.
    python scripts/dl_probe.py CONFIG N K"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from deppy_amd import _lib  # noqa: E402


def main():
    cfg, n, k = (int(x) for x in sys.argv[1:4])
    w = _lib.generate(cfg, n, 1)
    wa = _lib.WireArrays(**{x: w[x] for x in ("prob_var_off", "var_id", "var_con_off", "con_kind", "con_n",
                                               "con_arg_off", "con_arg", "str_off")}, str_bytes=w["str_bytes"].tobytes())
    ctx = _lib.Context(0, 1)
    dl = _lib.DeviceLowerer(ctx)
    w32 = _lib.Wire32Arrays(wa)
    lw = _lib.Lowered.empty()
    ts = []
    for _ in range(k):
        t0 = time.perf_counter()
        dl.lower(w32, lw)
        ts.append(time.perf_counter() - t0)
    host = _lib.Lowered(wa, narrow=True, pinned=True, packed=True)
    th = []
    for _ in range(k):
        t0 = time.perf_counter()
        host.relower(wa)
        th.append(time.perf_counter() - t0)
    same = np.array_equal(lw.rec, host.rec) and np.array_equal(lw.ident_var, host.ident_var)
    print("config %d n %d: device %.3f ms (min %.3f) host-lowered %d, host %.3f ms, wire %.1f MB, records %.1f MB, "
          "identities %.1f MB, equal %s" % (cfg, n, 1e3 * np.median(ts), 1e3 * min(ts), dl.host_count,
                                            1e3 * np.median(th), w32.nbytes() / 1e6, 4 * lw.rec_off[-1] / 1e6,
                                            8 * lw.ident_off[-1] / 1e6, same), flush=True)
    dl.close()
    ctx.close()


if __name__ == "__main__":
    main()
