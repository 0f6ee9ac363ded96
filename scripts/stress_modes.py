"""Repeat forced multi-wave solves (with and without tracing) against the
oracle to catch intermittent cross-wave races.  One process on the GPU box.

usage: python scripts/stress_modes.py <reps>
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402
from oracle import oracle  # noqa: E402  (checker only)
from tests.gpu_common import compare_results, lowered_config  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cases = [(5, 100, 53, 24), (5, 100, 52, 4096), (2, 400, 51, 0), (5, 120, 42, 0), (3, 500, 43, 0)]
ctxs = {f: _lib.Context(0, 1, flags=f) for f in (_lib.OPT_FORCE_GROUP, _lib.OPT_FORCE_HBM)}
bad_total = 0
for config, n, seed, cap in cases:
    lw = lowered_config(config, n, seed)
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16, trace_cap=cap) if cap else \
        oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    for f, c in ctxs.items():
        for r in range(reps):
            g = c.solve(lw.rec_off, lw.rec, cap)
            bad = compare_results(g, o, n)
            if cap:
                bad += [p for p in range(n) if not np.array_equal(
                    g["trace"][p][:g["trace_len"][p]], o["trace"][p][:o["trace_len"][p]])]
            bad_total += len(bad)
            if bad:
                print("config", config, "seed", seed, "cap", cap, "flags", f, "rep", r, "bad", bad[:3], flush=True)
    print("done", config, seed, cap, flush=True)
print("total mismatches", bad_total, flush=True)
sys.exit(1 if bad_total else 0)
