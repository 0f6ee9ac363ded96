"""Shared helpers for the -m gpu tests (run on the MI355X box)."""
import numpy as np

from deppy_amd import _lib


def lowered_config(config, n, seed):
    w = _lib.generate(config, n, seed)
    return _lib.Lowered(_lib.WireArrays(**{k: w[k] for k in (
        "prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off", "con_arg",
        "str_off")}, str_bytes=w["str_bytes"].tobytes()))


def compare_results(g, o, n, rec_off=None, rec=None):
    """Bit-exact comparison of GPU and oracle dp_result dicts; returns mismatches."""
    bad = []
    for p in range(n):
        if g["status"][p] != o["status"][p] or g["flags"][p] != o["flags"][p] \
                or g["steps"][p] != o["steps"][p]:
            bad.append((p, "status/flags/steps", int(g["status"][p]), int(o["status"][p]),
                        int(g["flags"][p]), int(o["flags"][p]), int(g["steps"][p]), int(o["steps"][p])))
            continue
        a0, a1 = g["inst_off"][p], g["inst_off"][p + 1]
        if not np.array_equal(g["installed"][a0:a1], o["installed"][a0:a1]):
            bad.append((p, "installed"))
            continue
        c0 = g["core_off"][p]
        cl = int(g["core_len"][p])
        if cl != o["core_len"][p] or not np.array_equal(g["core"][c0:c0 + cl], o["core"][c0:c0 + cl]):
            bad.append((p, "core"))
    return bad
