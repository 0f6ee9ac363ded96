"""Search trace (Tracer / SearchPosition, pkg/sat/tracer.go; Trace at every
unsatisfiable search step, pkg/sat/search.go:172-173).

The reference only logs traces (solve_test.go:302-353 writes them through
LoggingTracer and never asserts on them), and their Conflicts() come from
gini's Why, so trace content is parity-unpinned against the reference.  What
is pinned: the HIP kernel's event stream equals the oracle's (same events,
same order, same variables and identities) in every placement, tracing does
not change any result, and LoggingTracer's output format (tracer.go:26-35).
"""
import io

import numpy as np
import pytest

from deppy_amd import _lib, sat
from oracle import oracle
from tests import fixtures
from tests.gpu_common import compare_results, lowered_config
from tests.test_lowering import sat_var

CAP = 4096


@pytest.mark.parametrize("config,n,seed", [(2, 300, 5), (5, 120, 6)])
def test_oracle_trace_does_not_change_results(config, n, seed):
    lw = lowered_config(config, n, seed)
    a = oracle.solve_batch(lw.rec_off, lw.rec, 0, 8)
    b = oracle.solve_batch(lw.rec_off, lw.rec, 0, 8, trace_cap=CAP)
    for k in ("status", "steps", "core_len", "installed", "core"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["flags"], b["flags"] & ~_lib.F_TRACE_TRUNCATED)
    # every UNSAT problem that reached the search traced at least its final step
    searched = (b["status"] == -1) & ((b["flags"] & 0x10) == 0)
    assert (b["trace_len"][searched] > 0).all()


def test_oracle_trace_events_well_formed():
    lw = lowered_config(5, 80, 7)
    b = oracle.solve_batch(lw.rec_off, lw.rec, 0, 8, trace_cap=CAP)
    for p in range(lw.n):
        rec = lw.record(p)
        nv, nid = int(rec[1]), int(rec[6])
        for vs, ids in _lib.trace_events(b, p):
            assert all(0 <= v < nv for v in vs) and len(set(vs)) == len(vs)
            assert ids == sorted(set(ids)) and all(0 <= i < nid for i in ids)


def test_oracle_trace_truncation_is_clean():
    lw = lowered_config(5, 60, 8)
    full = oracle.solve_batch(lw.rec_off, lw.rec, 0, 8, trace_cap=1 << 16)
    small = oracle.solve_batch(lw.rec_off, lw.rec, 0, 8, trace_cap=16)
    for p in range(lw.n):
        ev_full = _lib.trace_events(full, p)
        ev_small = _lib.trace_events(small, p)
        # a truncated trace is a prefix of whole events
        assert ev_small == ev_full[:len(ev_small)]
        assert bool(small["flags"][p] & _lib.F_TRACE_TRUNCATED) == (len(ev_small) < len(ev_full))


# ---------------------------------------------------------------------------
# GPU: the kernel's event stream equals the oracle's
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("packed", [False, True], ids=["i32", "packed"])
@pytest.mark.parametrize("flags", [0, _lib.OPT_FORCE_GROUP, _lib.OPT_FORCE_HBM, _lib.OPT_FORCE_LDSG],
                         ids=["lds", "split", "hbm", "ldsg"])
@pytest.mark.parametrize("config,n,seed,cap", [(2, 400, 51, CAP), (5, 100, 52, CAP), (5, 100, 53, 24)])
def test_gpu_trace_bit_exact(config, n, seed, cap, flags, packed):
    """The kernel's trace equals the oracle's in every placement, from int32
    records and from packed ones (DP_FMT_P16D: the one-wavefront and M_LDSG
    kernels keep their bitsets over rows and map them back to identities for
    the trace, solve_kernel.hpp to_idents), the cap=24 truncation included."""
    lw = lowered_config(config, n, seed)
    src = lowered_config(config, n, seed, packed=True, pinned=True) if packed else lw
    c = _lib.Context(0, 1, flags=flags)
    try:
        g = c.solve(src.rec_off, src.rec, cap)
    finally:
        c.close()
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16, trace_cap=cap)
    assert compare_results(g, o, n) == []
    assert np.array_equal(g["flags"], o["flags"])
    assert np.array_equal(g["trace_len"], o["trace_len"])
    for p in range(n):
        assert np.array_equal(g["trace"][p][:g["trace_len"][p]], o["trace"][p][:o["trace_len"][p]]), p


@pytest.mark.gpu
def test_gpu_logging_tracer_format():
    """LoggingTracer through the sat API on the reference's UNSAT test cases."""
    cases = [c for c in fixtures.load("testsolve")["cases"] if c["error"] is not None]
    assert cases
    for case in cases:
        variables = [sat_var(v) for v in case["variables"]]
        out = io.StringIO()
        s, err = sat.NewSolver(sat.WithInput(variables), sat.WithTracer(sat.LoggingTracer(out)))
        assert err is None
        _, err = s.Solve(None)
        assert isinstance(err, sat.NotSatisfiable)
        text = out.getvalue()
        blocks = text.split("---\n")[1:]
        names = {str(v.Identifier()) for v in variables}
        for b in blocks:  # tracer.go:26-35
            head, _, conf = b.partition("Conflicts:\n")
            assert head.startswith("Assumptions:\n")
            for line in head.splitlines()[1:]:
                assert line.startswith("- ") and line[2:] in names
            for line in conf.splitlines():
                assert line.startswith("- ")


@pytest.mark.gpu
def test_gpu_tracer_events_match_oracle_through_api():
    """A recording tracer sees exactly the oracle's events, mapped to Variables
    and AppliedConstraints (lit_mapping.go:198-207 mapping)."""
    w = _lib.generate(5, 40, 61)
    inputs = []
    lw = lowered_config(5, 40, 61)
    for p in range(lw.n):
        inputs.append(fixtures.wire_problem_variables(w, p))

    class Rec(sat.Tracer):
        def __init__(self):
            self.events = []

        def Trace(self, pos):
            self.events.append(([str(v.Identifier()) for v in pos.Variables()],
                                [str(a) for a in pos.Conflicts()]))

    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16, trace_cap=1 << 16)
    for p in range(lw.n):
        t = Rec()
        sat.SolveBatch([inputs[p]], tracer=t)
        variables = inputs[p]
        i0 = int(lw.ident_off[p])
        expect = []
        for vs, ids in _lib.trace_events(o, p):
            conf = []
            for i in ids:
                var = variables[int(lw.ident_var[i0 + i])]
                conf.append(str(sat.AppliedConstraint(var, var.Constraints()[int(lw.ident_con[i0 + i])])))
            expect.append(([str(variables[v].Identifier()) for v in vs], conf))
        assert t.events == expect, p


@pytest.mark.gpu
def test_tracer_that_solves_inside_trace():
    """A Tracer whose Trace calls SolveBatch on the same thread: the nested
    call lowers into its own storage, so the outer batch's cores and trace
    still map to its own identities (sat.py _reused_lowered)."""
    w = _lib.generate(5, 30, 71)
    inputs = [fixtures.wire_problem_variables(w, p) for p in range(30)]
    plain = sat.SolveBatch(inputs)

    class Nested(sat.Tracer):
        def __init__(self):
            self.n = 0

        def Trace(self, pos):
            self.n += 1
            sat.SolveBatch(inputs[:3])  # another batch lowered while the outer one is mapped

    t = Nested()
    traced = sat.SolveBatch(inputs, tracer=t)
    assert t.n > 0
    for (ia, ea), (ib, eb) in zip(plain, traced):
        assert (ia is None) == (ib is None)
        if ia is not None:
            assert [v.Identifier() for v in ia] == [v.Identifier() for v in ib]
        assert type(ea) is type(eb) and str(ea) == str(eb)
