"""pkg/constraints: the sat.Variable implementation and the generator
aggregator that feed the solver (constraint_generator.go:11-40, variable.go:8-30)."""
from __future__ import annotations

from . import sat


class Variable(sat.Variable):
    """variable.go:10-30"""

    def __init__(self, id, *constraints):
        self.id = sat.Identifier(id)
        self.constraints = list(constraints)

    def Identifier(self) -> sat.Identifier:
        return self.id

    def Constraints(self) -> list:
        return self.constraints

    def AddConstraint(self, *constraint) -> None:
        self.constraints.extend(constraint)

    def __repr__(self):
        return "Variable(%r)" % str(self.id)


def NewVariable(id, *constraints) -> Variable:
    return Variable(id, *constraints)


class ConstraintGenerator:
    """constraint_generator.go:11-13"""

    def GetVariables(self, ctx, querier):  # pragma: no cover - interface
        raise NotImplementedError


class ConstraintAggregator(ConstraintGenerator):
    """constraint_generator.go:17-40: generators run in order, variables
    concatenated; the first error aborts."""

    def __init__(self, *generators):
        self.constraintGenerators = list(generators)

    def GetVariables(self, ctx, querier):
        variables: list = []
        for g in self.constraintGenerators:
            vs, err = g.GetVariables(ctx, querier)
            if err is not None:
                return None, err
            variables.extend(vs)
        return variables, None


def NewConstraintAggregator(*generators) -> ConstraintAggregator:
    return ConstraintAggregator(*generators)
