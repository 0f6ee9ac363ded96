"""pkg/solver: the resolution façade over pkg/sat (pkg/solver/solver.go:13-64).

    s, _ = NewDeppySolver(group, aggregator)
    solution, err = s.Solve(ctx)        # {EntityID: bool}

SolveBatch() resolves many (group, aggregator) pairs in one GPU launch — the
batch entry SURVEY.md §8(f) rank 2 asks for — with the same Solution
semantics per pair.
"""
from __future__ import annotations

from typing import Sequence

from . import sat
from .entitysource import EntityID


class Solution(dict):
    """solver.go:13-16: EntityID -> selected."""


class Solver:
    def Solve(self, ctx):  # pragma: no cover - interface
        raise NotImplementedError


class DeppySolver(Solver):
    """solver.go:22-64"""

    def __init__(self, entitySourceGroup, constraintAggregator):
        self.entitySourceGroup = entitySourceGroup
        self.constraintAggregator = constraintAggregator

    def Solve(self, ctx=None):
        return SolveBatch([self], ctx)[0]


def NewDeppySolver(entitySourceGroup, constraintAggregator):
    return DeppySolver(entitySourceGroup, constraintAggregator), None


def _solution(group, ctx, variables, selection) -> Solution:
    sol = Solution()
    for v in variables:  # every entity-backed variable starts false (solver.go:53-57)
        e = group.Get(ctx, EntityID(v.Identifier()))
        if e is not None:
            sol[e.ID()] = False
    for v in selection or []:  # then the selected ones are true (solver.go:58-62)
        e = group.Get(ctx, EntityID(v.Identifier()))
        if e is not None:
            sol[e.ID()] = True
    return sol


def SolveBatch(solvers: Sequence[DeppySolver], ctx=None) -> list:
    """[(Solution | None, error | None)] for each solver, one launch for all."""
    out: list = [None] * len(solvers)
    inputs, owners = [], []
    for i, d in enumerate(solvers):
        variables, err = d.constraintAggregator.GetVariables(ctx, d.entitySourceGroup)
        if err is not None:
            out[i] = (None, err)
            continue
        inputs.append(variables)
        owners.append(i)
    results = sat.SolveBatch(inputs) if inputs else []
    for variables, i, (selection, err) in zip(inputs, owners, results):
        if err is not None:  # NewSolver (duplicate) or Solve errors (solver.go:42-50)
            out[i] = (None, err)
        else:
            out[i] = (_solution(solvers[i].entitySourceGroup, ctx, variables, selection), None)
    return out
