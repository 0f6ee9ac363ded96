"""CPU restatement of deppy's lowering: []Variable -> lowered record.

TEST INFRASTRUCTURE ONLY (see oracle/sat_oracle.h): tests use it to check
the product's C++ lowering (deppy_amd/csrc/lower.cpp) record-for-record.

Restates
  * newLitMapping            pkg/sat/lit_mapping.go:40-77   (numbering, duplicate check,
                                                               constraints[m] last-writer-wins)
  * LitOf error accumulation pkg/sat/lit_mapping.go:81-88, 119-128
  * constraint Apply         pkg/sat/constraints.go:59-62 (Mandatory), :84-86 (Prohibited),
                             :116-123 (Dependency), :148-150 (Conflict), :180-186 (AtMost)
  * AnchorIdentifiers        pkg/sat/lit_mapping.go:163-174
  * Order() choice lists     pkg/sat/search.go:59-69, constraints.go:125-127
and, for the identity of each assumed constraint literal, the AND-inverter
graph of github.com/go-air/gini v1.0.4 `logic.C` (absent from /root/reference;
restated from its published behaviour): structural hashing of
And(a, b) with operands ordered, constant folding And(x,F)=F, And(x,T)=x,
And(x,x)=x, And(x,!x)=F; Or(a,b) = !And(!a,!b); CardSort = Batcher odd-even
merge sorting network over the inputs padded with F to a power of two,
comparator (a,b) -> (Or(a,b), And(a,b)); Leq(n) = F if n<0, T if n>=N, else
!sorted[n].
"""
from __future__ import annotations

import unicodedata

import numpy as np

MANDATORY, PROHIBITED, DEPENDENCY, CONFLICT, ATMOST = 1, 2, 3, 4, 5
REC_MAGIC = 0x31525044
H_SIZE = 16


# --------------------------------------------------------------------------
# Go %q (strconv.Quote) for error text
# --------------------------------------------------------------------------
_GO_ESC = {7: "\\a", 8: "\\b", 12: "\\f", 10: "\\n", 13: "\\r", 9: "\\t", 11: "\\v"}


def go_quote(b: bytes) -> str:
    out = ['"']
    i = 0
    while i < len(b):
        c = b[i]
        if c < 0x80:
            ch = chr(c)
            if ch in ('"', "\\"):
                out.append("\\" + ch)
            elif 0x20 <= c < 0x7F:
                out.append(ch)
            elif c in _GO_ESC:
                out.append(_GO_ESC[c])
            else:
                out.append("\\x%02x" % c)
            i += 1
            continue
        # multi-byte UTF-8
        n = 2 if c >> 5 == 6 else 3 if c >> 4 == 14 else 4 if c >> 3 == 30 else 0
        try:
            if n == 0:
                raise UnicodeDecodeError("utf-8", b, i, i + 1, "bad")
            ch = b[i:i + n].decode("utf-8")
        except UnicodeDecodeError:
            out.append("\\x%02x" % c)
            i += 1
            continue
        cp = ord(ch)
        if unicodedata.category(ch)[0] in "LMNPS":
            out.append(ch)
        elif cp < 0x10000:
            out.append("\\u%04x" % cp)
        else:
            out.append("\\U%08x" % cp)
        i += n
    out.append('"')
    return "".join(out)


# --------------------------------------------------------------------------
# AND-inverter graph with structural hashing (gini logic.C, recalled)
# --------------------------------------------------------------------------
F, T = 0, 1


class AIG:
    def __init__(self, n_inputs: int):
        self.next_node = 1 + n_inputs
        self.strash: dict[tuple[int, int], int] = {}

    @staticmethod
    def input(v: int) -> int:
        return 2 * (v + 1)

    def and_(self, a: int, b: int) -> int:
        if a == F or b == F:
            return F
        if a == T:
            return b
        if b == T:
            return a
        if a == b:
            return a
        if a == b ^ 1:
            return F
        if a > b:
            a, b = b, a
        g = self.strash.get((a, b))
        if g is None:
            g = 2 * self.next_node
            self.next_node += 1
            self.strash[(a, b)] = g
        return g

    def or_(self, a: int, b: int) -> int:
        return self.and_(a ^ 1, b ^ 1) ^ 1

    def cardsort(self, ms: list[int]) -> list[int]:
        n = len(ms)
        p = 1
        while p < n:
            p <<= 1
        a = list(ms) + [F] * (p - n)
        for i, j in batcher_pairs(p):
            hi, lo = self.or_(a[i], a[j]), self.and_(a[i], a[j])
            a[i], a[j] = hi, lo
        return a

    @staticmethod
    def leq(sorted_ms: list[int], n_inputs: int, b: int) -> int:
        if b < 0:
            return F
        if b >= n_inputs:
            return T
        return sorted_ms[b] ^ 1


def batcher_pairs(n: int) -> list[tuple[int, int]]:
    """Comparators of Batcher's odd-even merge sort for n = 2^k inputs."""
    pairs = []
    p = 1
    while p < n:
        k = p
        while k >= 1:
            for j in range(k % p, n - k, 2 * k):
                for i in range(min(k, n - j - k)):
                    if (i + j) // (2 * p) == (i + j + k) // (2 * p):
                        pairs.append((i + j, i + j + k))
            k //= 2
        p *= 2
    return pairs


# --------------------------------------------------------------------------
# lowering
# --------------------------------------------------------------------------
class Lowered:
    __slots__ = ("rec", "ident_var", "ident_con", "error", "msg")

    def __init__(self, rec, ident_var, ident_con, error=0, msg=None):
        self.rec = rec
        self.ident_var = ident_var
        self.ident_con = ident_con
        self.error = error  # 0 ok, 1 duplicate identifier, 2 lookup errors
        self.msg = msg


def lower_problem(variables) -> Lowered:
    """variables: list of (identifier: bytes, constraints: list of (kind, n, [bytes]))."""
    # pass 1, lit_mapping.go:50-57
    index: dict[bytes, int] = {}
    for i, (vid, _) in enumerate(variables):
        if vid in index:
            return Lowered(empty_record(), [], [], 1, "duplicate identifier %s in input" % go_quote(vid))
        index[vid] = i
    nv = len(variables)
    errs: list[str] = []

    def lit_of(x: bytes):
        v = index.get(x)
        if v is None:
            errs.append("variable %s referenced but not provided" % go_quote(x))
        return v

    aig = AIG(nv)
    key_ident: dict[int, int] = {}
    ident_owner: list[list[int]] = []
    clauses: list[tuple[list[int], int]] = []
    cards: list[tuple[list[int], int, int]] = []
    aux: list[int] = [nv]  # next auxiliary variable (AtMost network gates)

    # pass 2, lit_mapping.go:59-74
    for vi, (vid, cons) in enumerate(variables):
        s = vi
        for ci, (kind, n, args) in enumerate(cons):
            bad = False
            if kind == MANDATORY:
                m = aig.input(s)
            elif kind == PROHIBITED:
                m = aig.input(s) ^ 1
            elif kind == DEPENDENCY:
                m = aig.input(s) ^ 1
                for a in args:
                    d = lit_of(a)
                    if d is None:
                        bad = True
                        continue
                    m = aig.or_(m, aig.input(d))
            elif kind == CONFLICT:
                t = lit_of(args[0])
                if t is None:
                    bad = True
                else:
                    m = aig.or_(aig.input(s) ^ 1, aig.input(t) ^ 1)
            elif kind == ATMOST:
                ms = []
                for a in args:
                    d = lit_of(a)
                    if d is None:
                        bad = True
                        continue
                    ms.append(aig.input(d))
                if not bad:
                    m = AIG.leq(aig.cardsort(ms), len(ms), n)
            else:
                raise ValueError("unknown constraint kind %r" % kind)
            if bad or errs or m == T:
                continue
            ident = key_ident.get(m)
            if ident is None:
                ident = len(ident_owner)
                key_ident[m] = ident
                ident_owner.append([vi, ci])
                _emit_rows(m, nv, kind, s, n, args, index, ident, clauses, cards, aig, aux)
            else:
                ident_owner[ident] = [vi, ci]  # last writer wins, lit_mapping.go:69-72
    if errs:
        msg = "%d errors encountered: %s" % (len(errs), ", ".join(errs))
        return Lowered(empty_record(), [], [], 2, msg)

    # choices (Order()) and anchors
    var_choice_off = [0]
    choice_off = [0]
    choice_lits: list[int] = []
    anchors = []
    for vi, (vid, cons) in enumerate(variables):
        for kind, n, args in cons:
            if kind == DEPENDENCY and len(args) > 0:
                choice_lits.extend(index[a] for a in args)
                choice_off.append(len(choice_lits))
        var_choice_off.append(len(choice_off) - 1)
        if any(kind == MANDATORY for kind, _, _ in cons):
            anchors.append(vi)
    var_choice_off += [var_choice_off[-1]] * (aux[0] - nv)  # auxiliary variables: no choices
    rec = build_record(aux[0], clauses, cards, var_choice_off, choice_off, choice_lits, anchors,
                       len(ident_owner), nv if aux[0] > nv else 0)
    return Lowered(rec, [o[0] for o in ident_owner], [o[1] for o in ident_owner])


def _network_rows(m, nv, aig, ident, clauses, aux):
    """AtMost(n; ids) with an id listed more than once: the rows of the
    reference's own encoding, CardSort(ms).Leq(n) (constraints.go:180-186).
    Every And gate in the cone of the gate literal m gets an auxiliary
    variable (after the input's variables, in ascending node order) and its
    three Tseitin clauses [~g a] [~g b] [g ~a ~b]; then the unit [m].  Unit
    propagation over one such network derives what gini's does over its
    gates (the counting row is strictly stronger with repeated ids,
    DESIGN.md §3.1).  Each AtMost gets its own copy of its cone: two
    networks that share gates through the strash (the same ids with
    different bounds) share no auxiliary variable here, where gini has one
    variable per shared node -- a value forced on a shared gate by one
    network does not reach the other, so propagation can be weaker than
    gini's.  Sharing would need the gate rows always on (an identity's rows
    are dropped with it during core search).  Parity with the reference is
    unpinned for such inputs (no reference vector holds one).  Every row
    carries the AtMost's identity."""
    rev = {g: ab for ab, g in aig.strash.items()}
    cone, todo = set(), [m & ~1]
    while todo:
        g = todo.pop()
        if g in cone or g not in rev:
            continue
        cone.add(g)
        a, b = rev[g]
        todo += [a & ~1, b & ~1]
    var = {}
    for g in sorted(cone):
        var[g] = aux[0]
        aux[0] += 1

    def lit(x):  # AIG literal -> record literal (inputs: 2 * (node - 1))
        node = x >> 1
        v = node - 1 if 1 <= node <= nv else var[x & ~1]
        return 2 * v + (x & 1)

    for g in sorted(cone):
        a, b = rev[g]
        clauses.append(([lit(g) ^ 1, lit(a)], ident))
        clauses.append(([lit(g) ^ 1, lit(b)], ident))
        clauses.append(([lit(g), lit(a) ^ 1, lit(b) ^ 1], ident))
    clauses.append(([lit(m)], ident))


def _emit_rows(m, nv, kind, s, n, args, index, ident, clauses, cards, aig=None, aux=None):
    if m == F:
        clauses.append(([], ident))
        return
    node = m >> 1
    if 1 <= node <= nv:  # an input literal
        clauses.append(([2 * (node - 1) + (m & 1)], ident))
        return
    if kind == DEPENDENCY:
        lits = [2 * s + 1]
        for a in args:
            l = 2 * index[a]
            if l == 2 * s:
                return  # tautology: no row
            if l not in lits:
                lits.append(l)
        clauses.append((lits, ident))
    elif kind == CONFLICT:
        clauses.append(([2 * s + 1, 2 * index[args[0]] + 1], ident))
    elif kind == ATMOST:
        order: list[int] = []
        mult: dict[int, int] = {}
        for a in args:
            v = index[a]
            if v not in mult:
                order.append(v)
                mult[v] = 0
            mult[v] += 1
        if len(order) < len(args) and aig is not None:  # an id listed more than once
            _network_rows(m, nv, aig, ident, clauses, aux)
            return
        pos = [v for v in order for _ in range(mult[v])]
        cards.append((pos, n, ident))
    else:  # Mandatory / Prohibited always lower to an input literal
        raise AssertionError("unexpected gate literal for kind %d" % kind)


def build_record(nv, clauses, cards, var_choice_off, choice_off, choice_lits, anchors, nid, nvu=0):
    nc, nk = len(clauses), len(cards)
    clause_off = [0]
    clause_lits: list[int] = []
    for lits, _ in clauses:
        clause_lits.extend(lits)
        clause_off.append(len(clause_lits))
    card_off = [0]
    card_lits: list[int] = []
    for pos, _, _ in cards:
        card_lits.extend(pos)
        card_off.append(len(card_lits))
    body = (clause_off + clause_lits + [c[1] for c in clauses] + card_off + card_lits
            + [c[1] for c in cards] + [c[2] for c in cards] + var_choice_off + choice_off
            + choice_lits + anchors)
    hdr = [REC_MAGIC, nv, nc, nk, len(choice_off) - 1, len(anchors), nid, len(clause_lits),
           len(card_lits), len(choice_lits), 0, nvu, 0, 0, 0, 0]  # [11]: input variables when nv counts auxiliaries
    rec = np.array(hdr + body, dtype=np.int32)
    rec[10] = len(rec)
    return rec


def empty_record() -> np.ndarray:
    """Record of an errored problem (nv = 0)."""
    return build_record(0, [], [], [0], [0], [], [], 0)


# --------------------------------------------------------------------------
# wire format decoding (include/deppy_hip.h dp_wire) for the generator's output
# --------------------------------------------------------------------------
def problems_from_wire(w) -> list:
    """w: dict of numpy arrays named like dp_wire fields."""
    sb = w["str_bytes"]
    so = w["str_off"]

    def s(i):
        return bytes(sb[so[i]:so[i + 1]])

    out = []
    pvo, vid, vco = w["prob_var_off"], w["var_id"], w["var_con_off"]
    ck, cn, cao, ca = w["con_kind"], w["con_n"], w["con_arg_off"], w["con_arg"]
    for p in range(len(pvo) - 1):
        vs = []
        for v in range(pvo[p], pvo[p + 1]):
            cons = []
            for c in range(vco[v], vco[v + 1]):
                cons.append((int(ck[c]), int(cn[c]), [s(a) for a in ca[cao[c]:cao[c + 1]]]))
            vs.append((s(vid[v]), cons))
        out.append(vs)
    return out
