"""deppy_amd — MI355X-native batched dependency resolution (deppy pkg/sat).

    from deppy_amd import sat
    s, err = sat.NewSolver(sat.WithInput(variables))
    installed, err = s.Solve(None)

The engine is libdeppy_hip.so (C-ABI: include/deppy_hip.h), built in-tree by
deppy_amd/build.py.
"""
from . import sat  # noqa: F401

__all__ = ["sat"]
