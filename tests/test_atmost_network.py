"""AtMost rows that list a variable more than once: lowered as the reference's
own encoding, CardSort(ms).Leq(n) (pkg/sat/constraints.go:180-186), i.e.
gini's sorting network over auxiliary variables with its Tseitin rows
(lower.cpp Lowerer::network_rows, oracle/lower_ref.py _network_rows), so that
unit propagation over the record is unit propagation over gini's gates.  A
row listing every variable once keeps the counting row (the two propagate
alike there, tests/test_atmost_equivalence.py).

CPU: the product lowering equals the restatement record-for-record; the
record's network rows are exactly the Tseitin CNF the equivalence test builds
(the oracle matches the network restatement: same rows, and the oracle's unit
propagation over them derives what UP over the network derives); solved
records are semantically right by brute force (AtMost counts positions,
constraints.go:180-186: a SAT answer satisfies every constraint, an UNSAT
core is unsatisfiable by itself) and never install an auxiliary variable.
GPU: the kernel equals the oracle bit-for-bit on such catalogs in every
placement.  The reference's own tests hold no such row, so the installed sets
and cores are pinned by the restated algorithm, not by reference vectors.
"""
import itertools

import numpy as np
import pytest

from deppy_amd import _lib, sat
from oracle import lower_ref, oracle
from tests.test_atmost_equivalence import cnf, network, unit_propagate
from tests.test_lowering import V, compare

H_NV, H_NC, H_NID, H_NVU = 1, 2, 6, 11


def _ref(vs):
    return lower_ref.lower_problem([
        (v.Identifier().encode(), [(c.kind, c.n, [i.encode() for i in c.ids]) for c in v.Constraints()])
        for v in vs])


def _repeated_problems(seed, n_problems, max_vars=6):
    """Small random problems where most AtMosts list some variable twice or
    more, beside Dependencies, Conflicts, Mandatory and Prohibited."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_problems):
        nv = int(rng.integers(1, max_vars + 1))
        names = ["v%d" % i for i in range(nv)]
        vs = []
        for i in range(nv):
            cons = []
            for _ in range(int(rng.integers(0, 4))):
                k = int(rng.integers(1, 8))
                pick = lambda m: [names[j] for j in rng.integers(0, nv, m)]
                if k == 1:
                    cons.append(sat.Mandatory())
                elif k == 2:
                    cons.append(sat.Prohibited())
                elif k == 3:
                    cons.append(sat.Dependency(*pick(int(rng.integers(1, 4)))))
                elif k == 4:
                    cons.append(sat.Conflict(pick(1)[0]))
                else:
                    m = int(rng.integers(2, 7))
                    cons.append(sat.AtMost(int(rng.integers(0, m)), *pick(m)))
            vs.append(V(names[i], *cons))
        out.append(vs)
    return out


FIXED = [
    [V("a", sat.Mandatory()), V("b", sat.AtMost(1, "a", "a"))],           # a twice: ~a forced -> UNSAT
    [V("a"), V("b", sat.AtMost(1, "a", "a", "b"))],                       # ~a forced
    [V("a", sat.Dependency("b")), V("b"), V("u", sat.Mandatory(), sat.AtMost(2, "b", "b", "a"))],
    [V("a", sat.Mandatory(), sat.Dependency("b", "c")), V("b"), V("c"),
     V("u", sat.AtMost(2, "b", "c", "b", "a", "c"))],
    [V("x", sat.Mandatory(), sat.AtMost(3, "x", "y", "x", "y", "z", "x", "y", "z", "z")),
     V("y", sat.Mandatory()), V("z")],
]


def test_network_records_match_restatement():
    probs = FIXED + _repeated_problems(3, 300)
    lw = _lib.Lowered(sat.encode_inputs(probs))
    L = _lib.lib()
    n_net = 0
    for p, vs in enumerate(probs):
        ref = _ref(vs)
        compare(lw, p, ref)
        if ref.error:
            continue
        r = lw.record(p)
        assert L.dp_rec_validate(np.ascontiguousarray(r).ctypes.data_as(_lib.c_i32p), len(r)) == 0
        nvu = int(r[H_NVU])
        if nvu:
            n_net += 1
            assert nvu == len(vs) < int(r[H_NV])
    assert n_net > 100


def test_network_rows_are_the_tseitin_cnf():
    """The record of one AtMost(n; ids) with repeats holds exactly the
    Tseitin CNF of its network (test_atmost_equivalence.cnf, aux variables
    renumbered in ascending node order), every row with the AtMost's identity."""
    rng = np.random.default_rng(7)
    checked = 0
    for _ in range(60):
        V_ = int(rng.integers(1, 5))
        N = int(rng.integers(2, 9))
        ms = [int(v) for v in rng.integers(0, V_, N)]
        if len(set(ms)) == N:
            continue
        n = int(rng.integers(0, N))
        nv, gates, out = network(ms, n)
        if out == lower_ref.T or (out >> 1) <= nv:
            continue  # constant / input literal: no network rows
        names = ["v%d" % i for i in range(nv)]
        vs = [V(names[i]) for i in range(nv)] + [V("u", sat.AtMost(n, *[names[v] for v in ms]))]
        ref = _ref(vs)
        r = ref.rec
        nvr = int(r[H_NV])
        assert int(r[H_NVU]) == nv + 1
        # the expected CNF in record literals: input node k -> variable k-1, gate nodes in
        # ascending order -> nv+1, nv+2, ... (u is variable nv)
        exp = cnf(gates, out)
        gate_nodes = sorted({l >> 1 for c in exp for l in c if (l >> 1) > nv})
        ren = {g: nv + 1 + i for i, g in enumerate(gate_nodes)}
        assert nvr == nv + 1 + len(gate_nodes)

        def rl(l):
            node = l >> 1
            return 2 * (node - 1 if node <= nv else ren[node]) + (l & 1)
        want = sorted(sorted(rl(l) for l in c) for c in exp)
        nc = int(r[H_NC])
        off = 16
        clause_off = r[off:off + nc + 1]
        lits = r[off + nc + 1:off + nc + 1 + int(clause_off[-1])]
        ids = r[off + nc + 1 + int(clause_off[-1]):off + nc + 1 + int(clause_off[-1]) + nc]
        got = sorted(sorted(int(x) for x in lits[clause_off[i]:clause_off[i + 1]]) for i in range(nc))
        assert got == want, (ms, n)
        assert set(int(i) for i in ids) == {0} and int(r[3]) == 0  # one identity, no card row
        checked += 1
    assert checked > 15


def _model_ok(vs, x):
    """x: {name: bool} over the input's variables; the reference's semantics
    (constraints.go): AtMost counts positions."""
    for v in vs:
        s = v.Identifier()
        for c in v.Constraints():
            if c.kind == 1 and not x[s]:
                return False
            if c.kind == 2 and x[s]:
                return False
            if c.kind == 3 and x[s] and not any(x[d] for d in c.ids):
                return False
            if c.kind == 4 and x[s] and x[c.ids[0]]:
                return False
            if c.kind == 5 and sum(x[d] for d in c.ids) > c.n:
                return False
    return True


def _satisfiable(vs, keep=None):
    names = [v.Identifier() for v in vs]
    if keep is not None:
        vs = [V(v.Identifier(), *[c for j, c in enumerate(v.Constraints()) if (i, j) in keep])
              for i, v in enumerate(vs)]
    for bits in itertools.product((False, True), repeat=len(names)):
        if _model_ok(vs, dict(zip(names, bits))):
            return True
    return False


def test_oracle_on_network_records_is_semantically_right():
    probs = [p for p in FIXED + _repeated_problems(5, 400)]
    lw = _lib.Lowered(sat.encode_inputs(probs))
    res = oracle.solve_batch(lw.rec_off, lw.rec, 0, 8)
    n_sat = n_unsat = n_net = 0
    for p, vs in enumerate(probs):
        if lw.err[p]:
            continue
        r = lw.record(p)
        nvu = int(r[H_NVU]) or int(r[H_NV])
        n_net += int(r[H_NVU]) > 0
        st = int(res["status"][p])
        nvr = int(r[H_NV])
        inst_all = _lib.installed_list(res, p, nvr)
        assert all(v < nvu for v in inst_all), "an auxiliary variable installed"
        if st == 1:
            n_sat += 1
            on = set(inst_all)
            x = {v.Identifier(): i in on for i, v in enumerate(vs)}
            assert _model_ok(vs, x), p
        else:
            assert st == -1, st
            n_unsat += 1
            assert not _satisfiable(vs), p
            i0 = int(lw.ident_off[p])
            keep = set()
            for i in _lib.core_list(res, p):
                keep.add((int(lw.ident_var[i0 + i]), int(lw.ident_con[i0 + i])))
            assert not _satisfiable(vs, keep), p  # the core alone is unsatisfiable
    assert n_sat > 50 and n_unsat > 50 and n_net > 100, (n_sat, n_unsat, n_net)


def test_oracle_propagates_like_the_network():
    """Base propagation of AtMost(n; ms) with repeats plus units on some
    inputs (Mandatory / Prohibited): the oracle's verdict over the lowered
    record (UNSAT at the base, or the installed set when every input is fixed)
    equals unit propagation over the network restatement, which is weaker than
    counting here (test_atmost_equivalence: the deviation this lowering closes)."""
    rng = np.random.default_rng(11)
    stronger = 0
    for _ in range(150):
        V_ = int(rng.integers(1, 5))
        N = int(rng.integers(2, 8))
        ms = [int(v) for v in rng.integers(0, V_, N)]
        n = int(rng.integers(0, N))
        nv, gates, out = network(ms, n)
        if out == lower_ref.T:
            continue
        assign = {}
        for v in range(nv):
            x = rng.random()
            if x < 0.35:
                assign[v] = True
            elif x < 0.5:
                assign[v] = False
        names = ["v%d" % i for i in range(nv)]
        vs = []
        for i in range(nv):
            cons = [] if i not in assign else [sat.Mandatory() if assign[i] else sat.Prohibited()]
            vs.append(V(names[i], *cons))
        vs.append(V("u", sat.AtMost(n, *[names[v] for v in ms])))
        lw = _lib.Lowered(sat.encode_inputs([vs]))
        res = oracle.solve_batch(lw.rec_off, lw.rec, 0, 1)
        up = unit_propagate(cnf(gates, out), {v + 1: x for v, x in assign.items()})
        st = int(res["status"][0])
        # the record's base propagation is UP over exactly these rows and units
        if up is None:
            assert st == -1
            assert res["flags"][0] & 0x10  # DP_F_BASE_UNSAT
        else:
            assert not (res["flags"][0] & 0x10)
            counting_forced = {v for v in set(ms) if v not in assign and
                               sum(ms.count(w) for w in set(ms) if assign.get(w)) + ms.count(v) > n}
            up_forced = {v for v in set(ms) if v not in assign and (v + 1) in up}
            stronger += counting_forced != up_forced
    assert stronger > 0


def _catalogs_with_repeats(config, n, seed):
    """Generated catalogs (SURVEY §8(d) generator) with an AtMost that lists
    some package twice or more added to a few variables of each problem."""
    from tests import fixtures
    w = _lib.generate(config, n, seed)
    rng = np.random.default_rng(seed)
    out = []
    for p in range(n):
        vs = fixtures.wire_problem_variables(w, p)
        names = [v.Identifier() for v in vs]
        for _ in range(3):
            i = int(rng.integers(0, len(vs)))
            m = int(rng.integers(3, 9))
            ids = [names[int(j)] for j in rng.integers(0, len(vs), m - 1)]
            ids.append(ids[0])  # at least one repeat
            vs[i] = V(vs[i].Identifier(), *vs[i].Constraints(), sat.AtMost(int(rng.integers(1, 3)), *ids))
        out.append(vs)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, _lib.OPT_FORCE_GROUP, _lib.OPT_FORCE_MID, _lib.OPT_FORCE_HBM,
                                   _lib.OPT_FORCE_LDSG], ids=["lds", "split", "split4", "hbm", "ldsg"])
@pytest.mark.parametrize("form", ["i32", "narrow"])
def test_gpu_network_records_bit_exact(flags, form):
    """Repeated-id AtMosts lowered to network rows: the kernel equals the
    oracle bit-for-bit (status, flags, steps, installed set, core) in every
    placement, from int32 and from narrowed records, on small random problems
    and on generated catalogs; no auxiliary variable is ever installed."""
    probs = FIXED + _repeated_problems(21, 600) + _catalogs_with_repeats(2, 150, 22) \
        + _catalogs_with_repeats(5, 40, 23)
    lw = _lib.Lowered(sat.encode_inputs(probs), narrow=form == "narrow")
    nvu = np.array([int(lw.record(p)[H_NVU]) for p in range(lw.n)])
    assert (nvu > 0).sum() > 300
    c = _lib.Context(0, 1, flags=flags)
    try:
        g = c.solve(lw.rec_off, lw.rec)
    finally:
        c.close()
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    from tests.gpu_common import compare_results
    bad = compare_results(g, o, lw.n)
    assert bad == [], bad[:10]
    for p in np.flatnonzero(nvu > 0):
        nvr = int(lw.record(p)[H_NV])
        assert all(v < nvu[p] for v in _lib.installed_list(g, int(p), nvr))
    st = np.asarray(g["status"])
    assert (st == 1).sum() > 100 and (st == -1).sum() > 100


@pytest.mark.gpu
def test_gpu_network_through_sat_api():
    """The sat API on repeated-id problems: installed Variables and
    NotSatisfiable AppliedConstraints as the oracle's record maps them."""
    probs = FIXED + _repeated_problems(31, 200)
    out = sat.SolveBatch(probs)
    lw = _lib.Lowered(sat.encode_inputs(probs))
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 8)
    for p, vs in enumerate(probs):
        inst, err = out[p]
        if lw.err[p]:
            assert err is not None
            continue
        if int(o["status"][p]) == 1:
            assert err is None
            want = [vs[i].Identifier() for i in _lib.installed_list(o, p, len(vs))]
            assert [v.Identifier() for v in (inst or [])] == want
        else:
            assert isinstance(err, sat.NotSatisfiable)
            i0 = int(lw.ident_off[p])
            want = []
            for i in _lib.core_list(o, p):
                var = vs[int(lw.ident_var[i0 + i])]
                want.append(str(sat.AppliedConstraint(var, var.Constraints()[int(lw.ident_con[i0 + i])])))
            assert [str(a) for a in err] == want, p


def test_nvu_header_validated():
    """dp_rec_validate refuses an input-variable count outside 0..nv
    (DP_H_NVU, include/deppy_hip.h) and accepts the lowering's own."""
    lw = _lib.Lowered(sat.encode_inputs([FIXED[3]]))
    r = np.ascontiguousarray(lw.record(0)).copy()
    L = _lib.lib()
    nv = int(r[H_NV])
    assert 0 < int(r[H_NVU]) < nv
    for bad in (-1, nv + 1):
        r2 = r.copy()
        r2[H_NVU] = bad
        assert L.dp_rec_validate(r2.ctypes.data_as(_lib.c_i32p), len(r2)) == -21
    for ok in (0, nv):
        r2 = r.copy()
        r2[H_NVU] = ok
        assert L.dp_rec_validate(r2.ctypes.data_as(_lib.c_i32p), len(r2)) == 0


def test_two_networks_over_the_same_ids_get_their_own_gates():
    """Two repeated-id AtMosts over the same ids with different bounds share
    gates in gini's strash; here each lowers to its own copy of its cone
    (lower.cpp network_rows, lower_ref.py _network_rows): the record holds
    the auxiliaries of both networks side by side, the C++ lowering equals
    the restatement, and the oracle's answer satisfies both bounds.  Whether
    gini's shared gates would propagate more is parity-unpinned (no
    reference vector holds such a pair)."""
    vs = [V("a", sat.AtMost(1, "b", "b", "c"), sat.AtMost(2, "b", "b", "c"), sat.Mandatory()),
          V("b", sat.Mandatory()), V("c")]
    one = [V("a", sat.AtMost(1, "b", "b", "c"), sat.Mandatory()), V("b", sat.Mandatory()), V("c")]
    lw = _lib.Lowered(sat.encode_inputs([vs, one]))
    compare(lw, 0, _ref(vs))
    compare(lw, 1, _ref(one))
    r2, r1 = lw.record(0), lw.record(1)
    aux2, aux1 = int(r2[H_NV]) - int(r2[H_NVU]), int(r1[H_NV]) - int(r1[H_NVU])
    assert aux1 > 0 and aux2 > aux1  # the second network's gates are not the first one's
    res = oracle.solve_batch(lw.rec_off, lw.rec)
    assert list(res["status"]) == [-1, -1]  # b twice with b mandatory exceeds AtMost(1); a mandatory
