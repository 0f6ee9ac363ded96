"""AtMost propagation: gini's sorting-network encoding vs the kernel's counting.

The reference lowers AtMost(n, ids...) to CardSort(ms).Leq(n)
(pkg/sat/constraints.go:180-186): a Batcher odd-even merge network built in
gini's structurally hashed And-inverter graph, whose output is assumed and
propagated by gini's unit propagation over the Tseitin CNF of the gates.  The
kernel (and oracle/sat_oracle.c) instead propagate the row natively by
counting: count(true) > n is a conflict; a variable listed m times whose
m positions would push the count over n is forced false.

Class-A parity (A.6.2) rests on the two propagating exactly the same input
literals and conflicts.  This test checks it: it builds the network with the
restated AIG of oracle/lower_ref.py (the lowering oracle: constant folding,
And(x,x)=x, operand-ordered structural hashing), Tseitin-encodes its gates,
asserts the Leq(n) literal, and compares unit propagation from random partial
assignments of the inputs with the counting rule -- including inputs listed
more than once (multiplicity) and every bound 0 <= n < N.
"""
import itertools

import numpy as np
import pytest

from oracle import lower_ref

F, T = lower_ref.F, lower_ref.T


def network(ms_vars, n):
    """AIG of AtMost(n; ms_vars) over inputs 0..V-1 -> (gates, out literal)."""
    nv = max(ms_vars) + 1
    aig = lower_ref.AIG(nv)
    ms = [aig.input(v) for v in ms_vars]
    out = lower_ref.AIG.leq(aig.cardsort(ms), len(ms), n)
    gates = {g: pair for pair, g in aig.strash.items()}  # node literal -> (a, b)
    return nv, gates, out


def cnf(gates, out):
    """Tseitin clauses of the gates in the cone of `out`, plus the unit (out).
    Literals are AIG literals (2*node + neg); constants F=0/T=1."""
    clauses, todo, seen = [], [out & ~1], set()
    while todo:
        g = todo.pop()
        if g in seen or g not in gates:
            continue
        seen.add(g)
        a, b = gates[g]
        clauses += [[g ^ 1, a], [g ^ 1, b], [g, a ^ 1, b ^ 1]]
        todo += [a & ~1, b & ~1]
    clauses.append([out])
    return clauses


def unit_propagate(clauses, assign):
    """assign: {aig var node: bool}.  Returns None on conflict, else the fixpoint."""
    val = dict(assign)
    val[0] = False  # node 0: F (literal 0 false, literal 1 = T true)

    def lv(l):
        x = val.get(l >> 1)
        return None if x is None else (x != bool(l & 1))

    changed = True
    while changed:
        changed = False
        for c in clauses:
            unk, sat = [], False
            for l in c:
                x = lv(l)
                if x is True:
                    sat = True
                    break
                if x is None:
                    unk.append(l)
            if sat:
                continue
            if not unk:
                return None
            if len(unk) == 1:
                l = unk[0]
                val[l >> 1] = not bool(l & 1)
                changed = True
    return val


def counting(ms_vars, n, assign):
    """The kernel's rule (solve_kernel.hpp flush_cards; oracle eval_row)."""
    mult = {}
    for v in ms_vars:
        mult[v] = mult.get(v, 0) + 1
    cnt = sum(m for v, m in mult.items() if assign.get(v) is True)
    if cnt > n:
        return None
    forced = {v for v, m in mult.items() if assign.get(v) is None and cnt + m > n}
    return forced


def check(ms_vars, n, rng, trials, exact=True):
    """exact: UP over the network and counting derive the same literals; else
    (inputs listed more than once) the same conflicts and UP's implications a
    subset of counting's.  Returns the number of assignments where counting
    derived more."""
    nv, gates, out = network(ms_vars, n)
    if out == T:
        return 0  # trivially satisfied: no row
    clauses = cnf(gates, out)
    distinct = sorted(set(ms_vars))
    stronger = 0
    for _ in range(trials):
        assign = {}
        for v in distinct:
            r = rng.random()
            if r < 0.3:
                assign[v] = True
            elif r < 0.5:
                assign[v] = False
        up = unit_propagate(clauses, {v + 1: x for v, x in assign.items()})
        want = counting(ms_vars, n, assign)
        if want is None:
            assert up is None, (ms_vars, n, assign)
            continue
        assert up is not None, (ms_vars, n, assign)
        derived = {v for v in distinct if v not in assign and (v + 1) in up}
        assert all(up[v + 1] is False for v in derived), (ms_vars, n, assign)
        if exact:
            assert derived == want, (ms_vars, n, assign, derived, want)
        else:
            assert derived <= want, (ms_vars, n, assign, derived, want)
            stronger += derived != want
    return stronger


@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 16])
def test_network_up_equals_counting_distinct(N):
    rng = np.random.default_rng(N)
    for n in range(0, N):
        check(list(range(N)), n, rng, trials=60)
        perm = list(rng.permutation(N))
        check([int(v) for v in perm], n, rng, trials=30)


@pytest.mark.parametrize("seed", range(6))
def test_network_up_vs_counting_multiplicity(seed):
    """Inputs listed several times count with multiplicity (AtMost(n, a, a, b)
    holds at most n *positions*): constraints.go:180-186 passes every id to
    CardSort, duplicates included.  Here the two propagations are NOT the
    same: both detect exactly the same conflicts, and every literal UP over
    the network derives, counting derives too, but counting also forces a
    variable whose multiplicity alone exceeds the room left (cnt + m > n),
    which UP over the network sees only in some network shapes (And(x,x)=x
    folds some of them).  So the lowering does not give such a row a counting
    row: it emits the network's Tseitin rows (tests/test_atmost_network.py,
    DESIGN.md §3.1); the tests above are why a row listing every id once keeps
    its counting row."""
    rng = np.random.default_rng(100 + seed)
    stronger = 0
    for _ in range(25):
        V = int(rng.integers(1, 5))
        N = int(rng.integers(2, 9))
        ms = [int(v) for v in rng.integers(0, V, N)]
        for n in range(0, N):
            stronger += check(ms, n, rng, trials=20, exact=False)
    assert stronger > 0  # the deviation is real, and this test sees it


def test_batcher_network_sorts():
    """0-1 principle: the comparator lists lower_ref and lower.cpp build are
    sorting networks (descending) for every power of two up to 16."""
    for p in (1, 2, 4, 8, 16):
        pairs = lower_ref.batcher_pairs(p)
        for bits in itertools.product((0, 1), repeat=p):
            a = list(bits)
            for i, j in pairs:
                a[i], a[j] = max(a[i], a[j]), min(a[i], a[j])
            assert a == sorted(bits, reverse=True), (p, bits)
