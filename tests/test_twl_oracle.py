"""The one-wavefront kernel's two-watched-literal variant (DP_TWL_LDS,
solve_kernel.hpp twl_row) claims that propagating through two watched
positions per clause row gives every round exactly the occurrence lists'
outcome (the same rows found unit or conflicting, hence the same lowest
implying rows, conflicts, cores, trails and step counts).  The oracle built
with the same watch rules (oracle/Makefile libsat_oracle_twl.so) must
therefore agree field for field with the plain oracle on every workload, and
it counts what the lists buy: watch entries visited and the 64-entry batches
a wavefront would take for them."""
import numpy as np
import pytest

from oracle import oracle
from oracle import lower_ref
from tests import fixtures
from tests.gpu_common import lowered_config

KEYS = ("status", "flags", "installed", "core", "core_len", "steps")


@pytest.mark.parametrize("config,n", [(2, 300), (3, 3000), (5, 60), (6, 300)])
def test_twl_oracle_matches_occurrence_lists(config, n):
    lw = lowered_config(config, n, 4242 + config)
    a = oracle.solve_batch(lw.rec_off, lw.rec, 0, 4)
    L = oracle.twl_lib()
    st = np.zeros(7, np.int64)
    L.oracle_twl_stats(st, 1)
    b = oracle.solve_batch(lw.rec_off, lw.rec, 0, 1, L=L)
    L.oracle_twl_stats(st, 1)
    for k in KEYS:
        assert np.array_equal(a[k], b[k]), k
    rounds, entries, batches, dyn, moves, occ_entries, occ_batches = (int(x) for x in st)
    assert rounds > 0 and dyn > 0 and moves > 0 and entries < occ_entries and batches <= occ_batches
    print("config %d: %d rounds; watch entries %d (occurrence lists %d), 64-entry batches %d (%d); "
          "%d two-watched visits, %d moves" % (config, rounds, entries, occ_entries, batches, occ_batches, dyn, moves))


def test_twl_oracle_goldens():
    """TestSolve's 19 cases and the README example (tests/golden)."""
    cases = fixtures.load("testsolve")["cases"] + fixtures.load("readme")["cases"]
    for case in cases:
        rec = np.ascontiguousarray(lower_ref.lower_problem(fixtures.to_problem(case["variables"])).rec, np.int32)
        off = np.array([0, len(rec)], np.int64)
        a = oracle.solve_batch(off, rec, 0, 1)
        b = oracle.solve_batch(off, rec, 0, 1, L=oracle.twl_lib())
        for k in KEYS:
            assert np.array_equal(a[k], b[k]), (case["name"], k)
