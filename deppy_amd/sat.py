"""The deppy `pkg/sat` API, backed by the MI355X engine.

Mirrors /root/reference/pkg/sat so callers (pkg/solver, entitysource users) and
tests read the same as the reference's:

    s, err = NewSolver(WithInput(variables), WithTracer(t))     # solve.go:121-146
    installed, err = s.Solve(ctx)                                 # solve.go:53-119

Errors are returned as values, as in Go: DuplicateIdentifier from NewSolver
(lit_mapping.go:52-54); NotSatisfiable (solve.go:18-30), ErrIncomplete
(solve.go:14) or a lookup error ("%d errors encountered: ...",
lit_mapping.go:119-128) from Solve.  Installed variables come back in input
order and are the caller's own Variable objects (lit_mapping.go:176-184).

Solve() lowers the input (C++ dp_lower), solves it on the GPU (dp_solve) and
maps the result back.  There is no CPU path: without the HIP library or an
MI355X, Solve raises RuntimeError.  SolveBatch() solves many inputs in one
launch — the data-parallel form this engine exists for.
"""
from __future__ import annotations

import contextlib
import io
import os
import threading
import warnings
from dataclasses import dataclass, field
from typing import Iterable, Optional, Sequence

import numpy as np

from . import _lib

MANDATORY, PROHIBITED, DEPENDENCY, CONFLICT, ATMOST = 1, 2, 3, 4, 5
SAT, UNSAT, INCOMPLETE, ERROR = 1, -1, 0, -2


# ---------------------------------------------------------------------------
# variable.go
# ---------------------------------------------------------------------------
class Identifier(str):
    """variable.go:5-16"""

    def String(self) -> str:
        return str(self)


def IdentifierFromString(s: str) -> Identifier:
    return Identifier(s)


class Variable:
    """variable.go:19-27: anything with Identifier() and Constraints()."""

    def Identifier(self) -> Identifier:  # pragma: no cover - interface
        raise NotImplementedError

    def Constraints(self) -> list:  # pragma: no cover - interface
        raise NotImplementedError


class zeroVariable(Variable):
    def Identifier(self):
        return Identifier("")

    def Constraints(self):
        return []


# ---------------------------------------------------------------------------
# constraints.go
# ---------------------------------------------------------------------------
def _ids(ids) -> tuple:
    return tuple(Identifier(i) for i in ids)


@dataclass(frozen=True)
class Constraint:
    """constraints.go:13-18.  Apply(c, lm, subject) is replaced by the C++
    lowering (deppy_amd/csrc/lower.cpp); String/Order/Anchor are as in Go."""
    kind: int
    ids: tuple = ()
    n: int = 0

    def String(self, subject) -> str:
        s = str(subject)
        if self.kind == MANDATORY:
            return "%s is mandatory" % s  # constraints.go:57
        if self.kind == PROHIBITED:
            return "%s is prohibited" % s  # :81
        if self.kind == DEPENDENCY:
            if not self.ids:
                return "%s has a dependency without any candidates to satisfy it" % s  # :108
            return "%s requires at least one of %s" % (s, ", ".join(self.ids))  # :110-114
        if self.kind == CONFLICT:
            return "%s conflicts with %s" % (s, self.ids[0])  # :145
        if self.kind == ATMOST:
            return "%s permits at most %d of %s" % (s, self.n, ", ".join(self.ids))  # :173-177
        return ""

    def Order(self) -> Optional[list]:
        """constraints.go:125-127; nil for every other kind."""
        if self.kind == DEPENDENCY:
            return list(self.ids)
        return None

    def Anchor(self) -> bool:
        return self.kind == MANDATORY  # constraints.go:68-70

    def __repr__(self):
        names = {MANDATORY: "Mandatory", PROHIBITED: "Prohibited", DEPENDENCY: "Dependency",
                 CONFLICT: "Conflict", ATMOST: "AtMost"}
        args = ([str(self.n)] if self.kind == ATMOST else []) + [repr(str(i)) for i in self.ids]
        return "%s(%s)" % (names.get(self.kind, "?"), ", ".join(args))


def Mandatory() -> Constraint:
    return Constraint(MANDATORY)


def Prohibited() -> Constraint:
    return Constraint(PROHIBITED)


def Dependency(*ids) -> Constraint:
    return Constraint(DEPENDENCY, _ids(ids))


def Conflict(id) -> Constraint:
    return Constraint(CONFLICT, (Identifier(id),))


def AtMost(n: int, *ids) -> Constraint:
    return Constraint(ATMOST, _ids(ids), int(n))


class zeroConstraint(Constraint):
    def __init__(self):
        super().__init__(0)


@dataclass(eq=False)
class AppliedConstraint:
    """constraints.go:43-52"""
    Variable: Variable
    Constraint: Constraint

    def String(self) -> str:
        return self.Constraint.String(self.Variable.Identifier())

    def __str__(self):
        return self.String()

    def __eq__(self, other):
        return (isinstance(other, AppliedConstraint) and _var_eq(self.Variable, other.Variable)
                and self.Constraint == other.Constraint)

    def __repr__(self):
        return "AppliedConstraint(%r, %r)" % (str(self.Variable.Identifier()), self.Constraint)


def _var_eq(a, b) -> bool:
    return (a is b) or (a.Identifier() == b.Identifier() and
                        list(a.Constraints()) == list(b.Constraints()))


# ---------------------------------------------------------------------------
# errors (solve.go:14-30, lit_mapping.go:12-16, 119-128)
# ---------------------------------------------------------------------------
class SatError(Exception):
    def Error(self) -> str:
        return str(self)


class NotSatisfiable(SatError):
    """A (deletion-minimal, verified) set of applied constraints that cannot
    hold together (solve.go:16-30)."""

    def __init__(self, applied: Iterable[AppliedConstraint] = ()):
        self.applied = list(applied)
        super().__init__(self.Error())

    def Error(self) -> str:
        msg = "constraints not satisfiable"
        if not self.applied:
            return msg
        return msg + ": " + ", ".join(a.String() for a in self.applied)

    def __str__(self):
        return self.Error()

    def __iter__(self):
        return iter(self.applied)

    def __len__(self):
        return len(self.applied)

    def __getitem__(self, i):
        return self.applied[i]

    def __eq__(self, other):
        if isinstance(other, NotSatisfiable):
            return self.applied == other.applied
        return NotImplemented

    def __hash__(self):
        return id(self)


class DuplicateIdentifier(SatError):
    def __init__(self, ident, msg: Optional[str] = None):
        self.identifier = Identifier(ident)
        super().__init__(msg or 'duplicate identifier "%s" in input' % ident)

    def __eq__(self, other):
        return isinstance(other, DuplicateIdentifier) and self.identifier == other.identifier

    def __hash__(self):
        return hash(self.identifier)


class _Incomplete(SatError):
    pass


ErrIncomplete = _Incomplete("cancelled before a solution could be found")


class LookupErrors(SatError):
    """The aggregate returned by LitMapping.Error() (lit_mapping.go:119-128)."""


class InternalError(SatError):
    pass


# ---------------------------------------------------------------------------
# tracer.go
# ---------------------------------------------------------------------------
class SearchPosition:
    def Variables(self) -> list:  # pragma: no cover - interface
        raise NotImplementedError

    def Conflicts(self) -> list:  # pragma: no cover - interface
        raise NotImplementedError


class Tracer:
    def Trace(self, p: SearchPosition) -> None:  # pragma: no cover - interface
        raise NotImplementedError


class DefaultTracer(Tracer):
    def Trace(self, p):
        pass


class LoggingTracer(Tracer):
    """tracer.go:22-35"""

    def __init__(self, Writer: io.TextIOBase):
        self.Writer = Writer

    def Trace(self, p):
        self.Writer.write("---\nAssumptions:\n")
        for v in p.Variables():
            self.Writer.write("- %s\n" % v.Identifier())
        self.Writer.write("Conflicts:\n")
        for a in p.Conflicts():
            self.Writer.write("- %s\n" % a)


# ---------------------------------------------------------------------------
# solver (solve.go:32-163)
# ---------------------------------------------------------------------------
# The process-wide context.  _ctx_lock is held for a whole solve on it, so
# set_device() cannot close the context while a SolveBatch is using it (the
# library serialises calls on one context anyway).
_ctx_lock = threading.RLock()
_ctx: Optional[_lib.Context] = None


def device_context() -> _lib.Context:
    """The process-wide device context (device 0 of HIP_VISIBLE_DEVICES unless
    set_device() chose another)."""
    global _ctx
    with _ctx_lock:
        if _ctx is None:
            _ctx = _lib.Context(_device[0], 1)
        return _ctx


_device = [0]


def set_device(ordinal: int, step_budget: int = 0) -> None:
    """Bind this process to one MI355X (one process per GPU).  Waits for a
    solve in progress on the previous context."""
    global _ctx
    with _ctx_lock:
        if _ctx is not None:
            _ctx.close()
        _device[0] = ordinal
        _ctx = _lib.Context(ordinal, 1, step_budget)


class _Input:
    __slots__ = ("variables", "err")

    def __init__(self, variables):
        self.variables = list(variables) if variables is not None else []
        self.err = None


def encode_inputs(inputs: Sequence[Sequence[Variable]]) -> _lib.WireArrays:
    """[]Variable per problem -> wire arrays (identifiers interned per batch)."""
    strs: dict = {}
    str_bytes = bytearray()
    str_off = [0]

    def sid(x) -> int:
        b = str(x).encode("utf-8", "surrogateescape")
        i = strs.get(b)
        if i is None:
            i = len(str_off) - 1
            strs[b] = i
            str_bytes.extend(b)
            str_off.append(len(str_bytes))
        return i

    pvo, vid, vco, ck, cn, cao, ca = [0], [], [0], [], [], [0], []
    for variables in inputs:
        for v in variables:
            vid.append(sid(v.Identifier()))
            cons = v.Constraints() or []
            for c in cons:
                ck.append(c.kind)
                cn.append(c.n)
                for a in c.ids:
                    ca.append(sid(a))
                cao.append(len(ca))
            vco.append(vco[-1] + len(cons))
        pvo.append(len(vid))
    return _lib.WireArrays(pvo, vid, vco, ck, cn, cao, ca, str_off, bytes(str_bytes), True)


class Solver:
    """solve.go:32-34"""

    def Solve(self, ctx=None):  # pragma: no cover - interface
        raise NotImplementedError


class _solver(Solver):
    def __init__(self):
        self.input: Optional[_Input] = None
        self.tracer: Optional[Tracer] = None

    def Solve(self, ctx=None):
        """Returns (installed []Variable in input order | None, error | None).
        ctx is accepted for signature parity; like the reference (solve.go:83)
        a single solve is not interruptible."""
        return SolveBatch([self.input.variables], tracer=self.tracer)[0]


def NewSolver(*options):
    """solve.go:121-129: options first, then defaults."""
    s = _solver()
    for opt in list(options) + _defaults:
        err = opt(s)
        if err is not None:
            return None, err
    return s, None


def WithInput(input: Sequence[Variable]):
    def opt(s: _solver):
        s.input = _Input(input)
        err = _duplicate(s.input.variables)
        return err
    return opt


def WithTracer(t: Tracer):
    def opt(s: _solver):
        s.tracer = t
        return None
    return opt


def _default_input(s: _solver):
    if s.input is None:
        s.input = _Input([])
    return None


def _default_tracer(s: _solver):
    if s.tracer is None:
        s.tracer = DefaultTracer()
    return None


_defaults = [_default_input, _default_tracer]


def _duplicate(variables) -> Optional[DuplicateIdentifier]:
    seen = set()
    for v in variables:
        i = v.Identifier()
        if i in seen:
            lw = _lib.Lowered(encode_inputs([variables]))  # the library formats %q
            return DuplicateIdentifier(i, lw.msg[0])
        seen.add(i)
    return None


class _Position(SearchPosition):
    """One unsatisfiable search step as the GPU recorded it (search.go:205-217)."""

    def __init__(self, variables: list, conflicts: list):
        self._v, self._c = variables, conflicts

    def Variables(self) -> list:
        return list(self._v)

    def Conflicts(self) -> list:
        return list(self._c)


# trace words reserved per problem (dp_upload_traced); a truncated trace is
# re-solved alone with a larger reservation
TRACE_CAP = 1 << 12
TRACE_CAP_MAX = 1 << 24


def _replay_trace(tracer: Tracer, variables: list, lw, p: int, res: dict, j: int) -> None:
    """Deliver the recorded steps to the tracer in search order (search.go:173)."""
    i0 = int(lw.ident_off[p])
    for vs, ids in _lib.trace_events(res, j):
        conflicts = []
        for ident in ids:
            var = variables[int(lw.ident_var[i0 + ident])]
            conflicts.append(AppliedConstraint(var, var.Constraints()[int(lw.ident_con[i0 + ident])]))
        tracer.Trace(_Position([variables[v] for v in vs], conflicts))


# Lowering storage reused by solve_wire, per calling thread: the records of
# the last batch (page-locked, packed) stay valid until that thread's next
# call.  The page-locked storage stays pinned at the size of the thread's
# largest batch until the thread exits or calls release_lowering().  A call
# made while the thread's SolveBatch is still mapping results (a Tracer that
# solves from Trace) lowers into fresh storage, so the outer batch's
# identities and errors are not overwritten.
_lowering = threading.local()
LOWER_FLAGS = dict(narrow=True, packed=True, pinned=True)  # DP_LOWER_NARROW | PACKED | PINNED


def _reused_lowered(wire: _lib.WireArrays) -> _lib.Lowered:
    if getattr(_lowering, "busy", 0) > 1:  # a SolveBatch inside this thread's SolveBatch
        return _lib.Lowered(wire, **LOWER_FLAGS)
    lw = getattr(_lowering, "lw", None)
    if lw is None:
        lw = _lowering.lw = _lib.Lowered(wire, **LOWER_FLAGS)
    else:
        lw.relower(wire)
    return lw


def release_lowering() -> None:
    """Free this thread's reused lowering storage (page-locked memory)."""
    _lowering.lw = None
    _lowering.pipe = None
    _lowering.dlw = None
    _lowering.dl = None


# With SUB_BATCH > 0, a batch of at least 2 * SUB_BATCH problems is lowered
# and solved in sub-batches of SUB_BATCH, pipelined: the host pool lowers
# sub-batch i + 1 while the GPU solves sub-batch i (_solve_pipelined).
# Measured on the box (config 2, 10k catalogs, scripts/pipe_timing.py): the
# whole batch lowers in 3.8 ms and solves in 2.0 ms (6.3 ms through
# solve_wire), yet the pipelined path took 8.4 ms with 2048-problem
# sub-batches, 11.8 ms with 4096 and 6.3 ms with 8192 -- the sub-batches'
# lowering and solving did not overlap, and each sub-batch pays a launch
# tail (profiles/r05_pipe_timing.txt).  Off by default (0); the tests run it
# for parity.  DEPPY_SUB_BATCH sets it.
SUB_BATCH = int(os.environ.get("DEPPY_SUB_BATCH", "0"))


def _device_lowered(w32: "_lib.Wire32Arrays", ctx: _lib.Context) -> _lib.Lowered:
    """dp_lower_device into this thread's reused storage (its own from the
    host path's), with a device lowering per context kept per thread."""
    dls = getattr(_lowering, "dl", None)
    if dls is None:
        dls = _lowering.dl = {}
    dl = dls.get(id(ctx))
    if dl is None or dl.ctx is not ctx:
        dl = dls[id(ctx)] = _lib.DeviceLowerer(ctx)
    lw = getattr(_lowering, "dlw", None)
    if lw is None:
        lw = _lowering.dlw = _lib.Lowered.empty(**LOWER_FLAGS)
    return dl.lower(w32, lw)


def solve_wire(wire, context: Optional[_lib.Context] = None, trace_cap: int = 0):
    """The shipped path of SolveBatch from the wire format to host results:
    dp_lower_into(NARROW | PACKED | PINNED) into this thread's reused,
    page-locked storage, then dp_solve on the batch as it lies (dp_submit +
    dp_job_wait; up to 16 catalogs on the latency path).  The records are the
    form the GPU reads and are DMA'd without staging (the bench's `value` and
    `end_to_end` legs time the same records).  Problems the lowering rejected
    keep an empty record, solved as nothing and reported from lw.err.  A
    large untraced batch goes through _solve_pipelined (the same records,
    lowered and solved in overlapping sub-batches).
    Returns (lowered, results); both stay valid until this thread's next
    call.  trace_cap > 0 solves through the traced device-resident form.
    A compact wire (_lib.Wire32Arrays, include/deppy_hip.h dp_wire32) is
    lowered on the GPU instead (dp_lower_device, the same records)."""
    if isinstance(wire, _lib.Wire32Arrays):
        with (contextlib.nullcontext() if context else _ctx_lock):
            ctx = context or device_context()
            lw = _device_lowered(wire, ctx)
            res = ctx.solve(lw.rec_off, lw.rec, trace_cap)
        return lw, res
    if trace_cap <= 0 and SUB_BATCH > 0 and wire.n_problems >= 2 * SUB_BATCH:
        return _solve_pipelined(wire, context)
    lw = _reused_lowered(wire)
    with (contextlib.nullcontext() if context else _ctx_lock):
        ctx = context or device_context()
        res = ctx.solve(lw.rec_off, lw.rec, trace_cap)
    return lw, res


class _Stitched:
    """The lowering outputs SolveBatch reads (identities, errors), gathered
    from the sub-batches of a pipelined solve (copies: the sub-batches'
    storage is reused)."""

    def __init__(self, parts):
        self.n = sum(x[0] for x in parts)
        offs = [0]
        for _, io, _, _, _, _ in parts:
            offs.append(offs[-1] + int(io[-1]))
        self.ident_off = np.concatenate([[0]] + [io[1:] + offs[k] for k, (_, io, _, _, _, _) in enumerate(parts)])
        self.ident_var = np.concatenate([x[2] for x in parts]) if parts else np.zeros(0, np.int32)
        self.ident_con = np.concatenate([x[3] for x in parts]) if parts else np.zeros(0, np.int32)
        self.err = np.concatenate([x[4] for x in parts]) if parts else np.zeros(0, np.int32)
        self.msg = [m for x in parts for m in x[5]]


def _stitch_results(rs: list) -> dict:
    """Per-sub-batch result dicts (result_arrays layout) -> one, in order."""
    out = {k: np.concatenate([r[k] for r in rs]) for k in ("status", "flags", "core_len", "steps")}
    for data, off in (("installed", "inst_off"), ("core", "core_off")):
        parts, offs, at = [], [np.zeros(1, np.int64)], 0
        for r in rs:
            o = r[off]
            parts.append(r[data][:int(o[-1])])
            offs.append(o[1:] + at)
            at += int(o[-1])
        out[data] = np.concatenate(parts) if at else np.zeros(1, rs[0][data].dtype)
        out[off] = np.concatenate(offs)
    return out


def _solve_pipelined(wire: _lib.WireArrays, context: Optional[_lib.Context]):
    n = wire.n_problems
    cuts = list(range(0, n, SUB_BATCH)) + [n]
    pipe = getattr(_lowering, "pipe", None)
    if pipe is None or getattr(_lowering, "busy", 0) > 1:
        pipe = [None, None]
        if getattr(_lowering, "busy", 0) <= 1:
            _lowering.pipe = pipe
    parts, results, jobs = [], [], []
    with (contextlib.nullcontext() if context else _ctx_lock):
        ctx = context or device_context()

        def collect():
            lw, job = jobs.pop(0)
            results.append(job.wait())
            parts.append((lw.n, lw.ident_off.copy(), lw.ident_var.copy(), lw.ident_con.copy(), lw.err.copy(),
                          list(lw.msg)))

        for i in range(len(cuts) - 1):
            if len(jobs) == 2:
                collect()  # frees the storage sub-batch i reuses
            sub = wire.slice(cuts[i], cuts[i + 1])
            k = i % 2
            if pipe[k] is None:
                pipe[k] = _lib.Lowered(sub, **LOWER_FLAGS)
            else:
                pipe[k].relower(sub)
            jobs.append((pipe[k], ctx.submit(pipe[k].rec_off, pipe[k].rec)))
        while jobs:
            collect()
    return _Stitched(parts), _stitch_results(results)


def SolveBatch(inputs: Sequence[Sequence[Variable]], tracer: Optional[Tracer] = None,
               context: Optional[_lib.Context] = None) -> list:
    """Solve many independent problems in one GPU launch.

    With a tracer other than DefaultTracer the GPU records every
    unsatisfiable search step and the steps are replayed through
    tracer.Trace, problem by problem, before this returns.

    Returns [(installed | None, error | None)] in input order."""
    inputs = [list(v) for v in inputs]
    traced = tracer is not None and not isinstance(tracer, DefaultTracer)
    out: list = [None] * len(inputs)
    if not inputs:
        return out
    _lowering.busy = getattr(_lowering, "busy", 0) + 1
    try:
        return _solve_batch(inputs, tracer, traced, context, out)
    finally:
        _lowering.busy -= 1


def _solve_batch(inputs, tracer, traced, context, out) -> list:
    lw, res = solve_wire(encode_inputs(inputs), context, TRACE_CAP if traced else 0)
    retraced = {}
    if traced:
        with (contextlib.nullcontext() if context else _ctx_lock):
            ctx = context or device_context()
            for p in range(len(inputs)):
                if lw.err[p]:
                    continue
                rj, jj, cap = res, p, TRACE_CAP
                while rj["flags"][jj] & _lib.F_TRACE_TRUNCATED and cap < TRACE_CAP_MAX:
                    cap *= 16
                    r1 = np.ascontiguousarray(lw.record(p))
                    rj, jj = ctx.solve(np.array([0, len(r1)], np.int64), r1, cap), 0
                if rj["flags"][jj] & _lib.F_TRACE_TRUNCATED:
                    # the reference's tracer sees every unsatisfiable step
                    # (search.go:173); this one would miss the steps past the
                    # largest reservation
                    warnings.warn("deppy_amd: search trace of problem %d truncated at %d words; "
                                  "the tracer sees only its first steps" % (p, TRACE_CAP_MAX),
                                  RuntimeWarning, stacklevel=2)
                retraced[p] = (rj, jj)
    for p in range(len(inputs)):
        variables = inputs[p]
        if lw.err[p] == 1:
            out[p] = (None, DuplicateIdentifier(_dup_id(variables), lw.msg[p]))
            continue
        if lw.err[p] == 2:
            out[p] = (None, LookupErrors(lw.msg[p]))
            continue
        if traced:
            rj, jj = retraced[p]
            _replay_trace(tracer, variables, lw, p, rj, jj)
        st = int(res["status"][p])
        if st == SAT:
            inst = _lib.installed_list(res, p, len(variables))
            out[p] = ([variables[v] for v in inst] or None, None)
        elif st == UNSAT:
            i0 = int(lw.ident_off[p])
            applied = []
            for ident in _lib.core_list(res, p):
                vi = int(lw.ident_var[i0 + ident])
                ci = int(lw.ident_con[i0 + ident])
                var = variables[vi]
                applied.append(AppliedConstraint(var, var.Constraints()[ci]))
            out[p] = (None, NotSatisfiable(applied))
        elif st == INCOMPLETE:
            out[p] = (None, ErrIncomplete)
        else:
            out[p] = (None, InternalError("unexpected internal error"))
    return out


def _dup_id(variables):
    seen = set()
    for v in variables:
        if v.Identifier() in seen:
            return v.Identifier()
        seen.add(v.Identifier())
    return Identifier("")
