"""Run one batch through one placement and compare with the oracle.

usage: python scripts/mode_probe.py <config> <n> <flags>   (flags: dp_opt_flag)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402
from oracle import oracle  # noqa: E402  (checker only)
from tests.gpu_common import compare_results, lowered_config  # noqa: E402

config, n, flags = (int(x) for x in sys.argv[1:4])
lw = lowered_config(config, n, 77)
ctx = _lib.Context(0, 1, flags=flags)
g = ctx.solve(lw.rec_off, lw.rec)
print("kernel ms %.3f" % ctx.last_kernel_ms(), flush=True)
o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
bad = compare_results(g, o, n)
print("config", config, "n", n, "flags", flags, "mismatches", len(bad), bad[:5],
      "status", np.unique(g["status"], return_counts=True), flush=True)
sys.exit(1 if bad else 0)
