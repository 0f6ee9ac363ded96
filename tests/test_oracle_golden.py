"""The CPU restatement (oracle/) against the reference's own test vectors.

This is what pins the oracle: TestSolve (19 cases), TestSearch (2 scripted
traces), TestDuplicateIdentifier and the README example, transcribed in
tests/golden/ (make_golden.py).
"""
import pytest

from oracle import lower_ref, oracle
from tests import fixtures

SOLVE = fixtures.load("testsolve")["cases"]
README = fixtures.load("readme")["cases"]


def run_case(case):
    lw = lower_ref.lower_problem(fixtures.to_problem(case["variables"]))
    assert lw.error == 0, lw.msg
    st, flags, installed, core, steps = oracle.solve(lw.rec)
    return lw, st, flags, installed, core


@pytest.mark.parametrize("case", SOLVE + README, ids=[c["name"] for c in SOLVE + README])
def test_solve_golden(case):
    variables = case["variables"]
    lw, st, flags, installed, core = run_case(case)
    if case["error"] is None:
        assert st == 1
        ids = sorted(variables[v]["id"] for v in installed)
        assert ids == (case["installed"] or [])
        # every golden SAT case is class A
        assert not flags & 2
    else:
        assert st == -1
        applied = [(lw.ident_var[i], lw.ident_con[i]) for i in core]
        got = fixtures.sorted_applied(variables, applied)
        assert got == case["error"]["applied"]
        assert fixtures.not_satisfiable_string(variables, got) == case["error"]["string"]


def test_core_is_verified_unsat():
    for case in SOLVE + README:
        if case["error"] is None:
            continue
        lw, st, flags, installed, core = run_case(case)
        assert oracle.refute(lw.rec, core) == -1
        for drop in core:  # deletion-minimal
            assert oracle.refute(lw.rec, [i for i in core if i != drop]) == 1


@pytest.mark.parametrize("case", fixtures.load("testsearch")["cases"],
                         ids=lambda c: c["name"])
def test_search_scripted(case):
    variables = case["variables"]
    lw = lower_ref.lower_problem(fixtures.to_problem(variables))
    res, lits, depth = oracle.search_scripted(lw.rec, case["test_returns"], case["untest_returns"])
    assert res == case["result"]
    got = [variables[v]["id"] for v in lits] or None
    assert got == case["assumptions"]
    assert depth == 0


def test_duplicate_identifier():
    e = fixtures.load("errors")["duplicate_identifier"]
    lw = lower_ref.lower_problem(fixtures.to_problem(e["variables"]))
    assert lw.error == 1 and lw.msg == e["string"]


def test_not_satisfiable_strings():
    for c in fixtures.load("errors")["not_satisfiable"]:
        applied = c["applied"] or []
        variables = [{"id": v, "constraints": [con]} for v, con in applied]
        sorted_ = [{"var": v, "constraint": 0} for v, _ in applied]
        assert fixtures.not_satisfiable_string(variables, sorted_) == c["string"]


def test_lookup_errors():
    vs = [{"id": "a", "constraints": [{"kind": "dependency", "ids": ["x", "b", "y"]}]},
          {"id": "b", "constraints": [{"kind": "conflict", "ids": ["z\"q"]}]}]
    lw = lower_ref.lower_problem(fixtures.to_problem(vs))
    assert lw.error == 2
    assert lw.msg == ('3 errors encountered: variable "x" referenced but not provided, '
                      'variable "y" referenced but not provided, '
                      'variable "z\\"q" referenced but not provided')


def test_order_golden():
    """TestOrder (pkg/sat/constraints_test.go:9-39): Order() per constraint
    kind, and the lowered record's choice lists are exactly the Order() lists
    of each variable's constraints, in constraint order (search.go:59-69)."""
    import numpy as np
    from deppy_amd import _lib, sat
    from tests.test_lowering import V, sat_var
    cases = fixtures.load("errors")["order"]
    assert [c["name"] for c in cases] == ["mandatory", "prohibited", "dependency", "conflict"]
    for c in cases:
        con = sat_var({"id": "s", "constraints": [c["constraint"]]}).Constraints()[0]
        got = con.Order()
        assert (None if got is None else [str(i) for i in got]) == c["expected"], c["name"]
    vs = [V("s", *[sat_var({"id": "s", "constraints": [c["constraint"]]}).Constraints()[0] for c in cases],
            sat.Dependency("c", "a")), V("a"), V("b"), V("c")]
    lw = _lib.Lowered(sat.encode_inputs([vs]))
    r = lw.record(0)
    L = {k: int(x) for k, x in zip(("nv", "nc", "nk", "nch", "na", "nid", "ncl", "nkl", "nchl"), r[1:10])}
    o = 16 + (L["nc"] + 1) + L["ncl"] + L["nc"] + (L["nk"] + 1) + L["nkl"] + 2 * L["nk"]
    var_choice_off = r[o:o + L["nv"] + 1]
    choice_off = r[o + L["nv"] + 1:o + L["nv"] + 1 + L["nch"] + 1]
    lits = r[o + L["nv"] + 1 + L["nch"] + 1:][:L["nchl"]]
    names = ["s", "a", "b", "c"]
    lists = [[names[int(v)] for v in lits[choice_off[k]:choice_off[k + 1]]]
             for k in range(var_choice_off[0], var_choice_off[1])]
    assert lists == [["a", "b", "c"], ["c", "a"]]
    assert np.all(np.diff(var_choice_off[1:]) == 0)
