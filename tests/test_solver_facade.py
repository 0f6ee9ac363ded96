"""pkg/solver + pkg/constraints + the entitysource lookups they use."""
import pytest

from deppy_amd import constraints, entitysource, sat, solver


class Gen(constraints.ConstraintGenerator):
    def __init__(self, vs=None, err=None):
        self.vs, self.err = vs or [], err

    def GetVariables(self, ctx, querier):
        return (None, self.err) if self.err else (list(self.vs), None)


def readme_setup():
    ents = {i: entitysource.NewEntity(i) for i in ("A-v0.1.0", "B-latest", "C-v0.1.0", "D-latest")}
    group = entitysource.NewGroup(entitysource.NewCacheQuerier(ents))
    v = constraints.NewVariable
    gens = [Gen([v("A-v0.1.0", sat.Mandatory(), sat.Dependency("C-v0.1.0")),
                 v("B-latest", sat.Mandatory(), sat.Dependency("D-latest"))]),
            Gen([v("C-v0.1.0"), v("D-latest"), v("E-unrelated")])]
    return group, constraints.NewConstraintAggregator(*gens)


def test_aggregator_order_and_errors():
    group, agg = readme_setup()
    vs, err = agg.GetVariables(None, group)
    assert err is None
    assert [str(x.Identifier()) for x in vs] == ["A-v0.1.0", "B-latest", "C-v0.1.0", "D-latest", "E-unrelated"]
    bad = constraints.NewConstraintAggregator(Gen([]), Gen(err=ValueError("boom")), Gen([]))
    assert isinstance(bad.GetVariables(None, group)[1], ValueError)


def test_group_first_source_wins():
    a = entitysource.NewCacheQuerier({"x": entitysource.NewEntity("x", {"src": "a"})})
    b = entitysource.NewCacheQuerier({"x": entitysource.NewEntity("x", {"src": "b"}),
                                      "y": entitysource.NewEntity("y")})
    g = entitysource.NewGroup(a, b)
    assert g.Get(None, "x").GetProperty("src") == ("a", None)
    assert g.Get(None, "y").ID() == "y" and g.Get(None, "z") is None
    assert str(g.Get(None, "y").GetProperty("nope")[1]) == "Property '(nope)' Not Found"


def test_generator_error_short_circuits_before_the_gpu():
    group, _ = readme_setup()
    s, _ = solver.NewDeppySolver(group, constraints.NewConstraintAggregator(Gen(err=KeyError("k"))))
    sol, err = s.Solve(None)
    assert sol is None and isinstance(err, KeyError)


@pytest.mark.gpu
def test_readme_solution():
    group, agg = readme_setup()
    s, _ = solver.NewDeppySolver(group, agg)
    sol, err = s.Solve(None)
    assert err is None
    # entity-backed variables default false, the selection true (solver.go:52-62);
    # E-unrelated has no entity, so it is absent
    assert sol == {"A-v0.1.0": True, "B-latest": True, "C-v0.1.0": True, "D-latest": True}


@pytest.mark.gpu
def test_batch_of_solvers():
    group, agg = readme_setup()
    v = constraints.NewVariable
    unsat = constraints.NewConstraintAggregator(Gen([v("A-v0.1.0", sat.Mandatory(), sat.Prohibited())]))
    out = solver.SolveBatch([solver.DeppySolver(group, agg), solver.DeppySolver(group, unsat)])
    assert out[0][1] is None and out[0][0]["D-latest"] is True
    assert out[1][0] is None and isinstance(out[1][1], sat.NotSatisfiable)
