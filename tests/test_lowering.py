"""Host logic on CPU: the product's C++ lowering (dp_lower) equals the
restatement in oracle/lower_ref.py record-for-record, and the library exports
every symbol include/deppy_hip.h declares."""
import ctypes
import re

import numpy as np
import pytest

from deppy_amd import _lib, sat
from oracle import lower_ref
from tests import fixtures

ROOT = fixtures.GOLDEN.rsplit("/tests/", 1)[0]


def test_exports_match_header():
    hdr = open(ROOT + "/include/deppy_hip.h").read()
    inline = set(re.findall(r"static inline [^(]*\b(dp_[a-z_0-9]+)\s*\(", hdr))
    declared = set(re.findall(r"\b(dp_[a-z_0-9]+)\s*\(", hdr)) - inline
    assert "dp_rec_layout_of" in inline
    assert declared == set(_lib.EXPORTS)
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert hasattr(L, name), name


def test_library_built_from_this_tree():
    """Build provenance: the library carries the digest of the sources,
    headers and flags it was compiled from (dp_build_info), equal to this
    tree's; a library whose digest differs is refused at load."""
    from deppy_amd import build
    info = _lib.build_info()
    assert info == "sources=%s arch=gfx950" % build.sources_digest(), info
    # a different tree (one more flag) would not match: the binding's check is live
    assert build.sources_digest(["-DDP_STAMPS"]) != build.sources_digest()


def test_stale_library_is_refused(monkeypatch):
    """A product library whose embedded digest is not the tree's raises at
    load instead of running (the sources changed since it was built)."""
    from deppy_amd import build
    L = ctypes.CDLL(_lib.LIB_PATH)
    monkeypatch.setattr(build, "sources_digest", lambda extra=None: "0123456789abcdef")
    with pytest.raises(RuntimeError, match="built from other sources"):
        _lib._check_provenance(L)


def variables_of(fixture_vars):
    return [sat_var(v) for v in fixture_vars]


class V(sat.Variable):
    def __init__(self, ident, *cons):
        self.ident = sat.Identifier(ident)
        self.cons = list(cons)

    def Identifier(self):
        return self.ident

    def Constraints(self):
        return self.cons


def sat_var(v):
    cons = []
    for c in v["constraints"]:
        k = c["kind"]
        if k == "mandatory":
            cons.append(sat.Mandatory())
        elif k == "prohibited":
            cons.append(sat.Prohibited())
        elif k == "dependency":
            cons.append(sat.Dependency(*c["ids"]))
        elif k == "conflict":
            cons.append(sat.Conflict(c["ids"][0]))
        else:
            cons.append(sat.AtMost(c["n"], *c["ids"]))
    return V(v["id"], *cons)


def all_golden_variable_sets():
    out = []
    for name in ("testsolve", "readme", "testsearch"):
        out += [c["variables"] for c in fixtures.load(name)["cases"]]
    return out


def compare(lw_product, p, ref):
    assert lw_product.err[p] == ref.error, (lw_product.msg[p], ref.msg)
    if ref.error:
        assert lw_product.msg[p] == ref.msg
        return
    np.testing.assert_array_equal(lw_product.record(p), ref.rec)
    i0, i1 = lw_product.ident_off[p], lw_product.ident_off[p + 1]
    assert list(lw_product.ident_var[i0:i1]) == list(ref.ident_var)
    assert list(lw_product.ident_con[i0:i1]) == list(ref.ident_con)


def test_golden_records_match_restatement():
    sets = all_golden_variable_sets()
    lw = _lib.Lowered(sat.encode_inputs([variables_of(vs) for vs in sets]))
    for p, vs in enumerate(sets):
        compare(lw, p, lower_ref.lower_problem(fixtures.to_problem(vs)))
        assert _lib.lib().dp_rec_validate(
            lw.record(p).ctypes.data_as(_lib.c_i32p), len(lw.record(p))) == 0


EDGE = [
    # identities that collide (lit_mapping.go:69-72): last writer is reported
    [V("a", sat.Conflict("b")), V("b", sat.Conflict("a"), sat.AtMost(1, "a", "b"))],
    [V("a", sat.Prohibited(), sat.Dependency(), sat.Conflict("a"), sat.AtMost(0, "a"))],
    [V("a", sat.Mandatory(), sat.Mandatory()), V("b", sat.AtMost(1, "b", "b"))],
    # tautologies and constants
    [V("a", sat.Dependency("a", "b")), V("b", sat.Dependency("c", "b")), V("c"),
     V("d", sat.AtMost(-1, "a")), V("e", sat.AtMost(3, "a", "b"))],
    # duplicates inside rows, multiplicity in AtMost
    [V("a", sat.Mandatory(), sat.Dependency("b", "b", "c")), V("b"), V("c"),
     V("u", sat.AtMost(2, "b", "c", "b", "a", "c"))],
    # empty problem, empty constraint lists
    [],
    [V("x"), V("y", sat.AtMost(0))],
    # errors: lookups accumulate in Apply order, %q quoting
    [V("a", sat.Dependency("nope", "b"), sat.AtMost(1, "zz")), V("b", sat.Conflict('q"\\\n\x01é '))],
    [V("a"), V("b"), V("a")],
]


def test_edge_records_match_restatement():
    lw = _lib.Lowered(sat.encode_inputs(EDGE))
    for p, vs in enumerate(EDGE):
        ref = lower_ref.lower_problem([
            (v.Identifier().encode(), [(c.kind, c.n, [i.encode() for i in c.ids]) for c in v.Constraints()])
            for v in vs])
        compare(lw, p, ref)


@pytest.mark.parametrize("config", [2, 3, 5])
def test_generated_records_match_restatement(config):
    w = _lib.generate(config, 40, 1234)
    lw = _lib.Lowered(_lib.WireArrays(**{k: w[k] for k in (
        "prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off", "con_arg",
        "str_off")}, str_bytes=w["str_bytes"].tobytes()))
    probs = lower_ref.problems_from_wire(w)
    for p, prob in enumerate(probs):
        compare(lw, p, lower_ref.lower_problem(prob))


def test_generator_is_deterministic():
    a = _lib.generate(2, 5, 77)
    b = _lib.generate(2, 5, 77)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])
    c = _lib.generate(2, 5, 78)
    assert not np.array_equal(a["con_arg"][:50], c["con_arg"][:50]) or len(a["con_arg"]) != len(c["con_arg"])


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(RuntimeError):
        _lib.Context(0, 1)


def test_device_bytes_16bit_form():
    """LDS-path records are read in 16-bit form (64 header bytes + 2 per
    word, or a packed record as it is); forcing the multi-wave path reads the
    int32 form (4 bytes per word; the watch lists it builds or brings are
    derived data, not algorithmic bytes)."""
    from tests.gpu_common import lowered_config
    lw = lowered_config(2, 50, 1000)
    off, rec = np.asarray(lw.rec_off), np.asarray(lw.rec)
    words = off[1:] - off[:-1]
    rb, ib = _lib.device_bytes(off, rec)
    assert rb == int((64 + 2 * (words - 16)).sum())
    assert ib > rb
    rb32, ib32 = _lib.device_bytes(off, rec, flags=1)  # DP_OPT_FORCE_GROUP
    assert rb32 == 4 * int(words.sum()) and ib32 > ib
    pk = lowered_config(2, 50, 1000, packed=True)
    rbp, _ = _lib.device_bytes(pk.rec_off, pk.rec)
    assert rbp <= 4 * int(np.diff(pk.rec_off).sum()) and rbp < 0.8 * rb


def _random_problems(seed, n_problems, max_vars=7):
    """Small random problems over a tiny identifier alphabet: identity
    collisions (Conflict vs AtMost(1;a,b), AtMost(0;a,b) pairs, Prohibited vs
    Dependency()/Conflict(v,v)/AtMost(0;v), repeated Dependencies, AtMosts over
    one set in one or two orders, multiplicities) are frequent."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_problems):
        nv = int(rng.integers(1, max_vars + 1))
        names = ["v%d" % i for i in range(nv)]
        vs = []
        for i in range(nv):
            cons = []
            for _ in range(int(rng.integers(0, 5))):
                k = int(rng.integers(1, 6))
                pick = lambda m: [names[j] for j in rng.integers(0, nv, m)]
                if k == 1:
                    cons.append(sat.Mandatory())
                elif k == 2:
                    cons.append(sat.Prohibited())
                elif k == 3:
                    cons.append(sat.Dependency(*pick(int(rng.integers(0, 4)))))
                elif k == 4:
                    cons.append(sat.Conflict(pick(1)[0]))
                else:
                    m = int(rng.integers(0, 5))
                    ids = pick(m) if rng.random() < 0.3 else list(rng.permutation(names)[:m])
                    cons.append(sat.AtMost(int(rng.integers(-1, m + 1)), *ids))
            vs.append(V(names[i], *cons))
        out.append(vs)
    return out


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_fast_lowering_equals_exact_aig(seed, monkeypatch):
    """The key-based identity path (lower_fast) is record-for-record equal to
    the full And-inverter graph (lower_one) and to oracle/lower_ref.py."""
    probs = _random_problems(seed, 400)
    wire = sat.encode_inputs(probs)
    fast = _lib.Lowered(wire)
    monkeypatch.setenv("DEPPY_LOWER_EXACT", "1")
    exact = _lib.Lowered(wire)
    assert exact.n_exact == len(probs)
    # most problems take the key path, collisions included
    assert fast.n_exact < 0.5 * len(probs), fast.n_exact
    np.testing.assert_array_equal(fast.rec_off, exact.rec_off)
    np.testing.assert_array_equal(fast.rec, exact.rec)
    np.testing.assert_array_equal(fast.ident_var, exact.ident_var)
    np.testing.assert_array_equal(fast.ident_con, exact.ident_con)
    assert fast.msg == exact.msg
    for p, vs in enumerate(probs[:120]):
        ref = lower_ref.lower_problem([
            (v.Identifier().encode(), [(c.kind, c.n, [i.encode() for i in c.ids]) for c in v.Constraints()])
            for v in vs])
        compare(fast, p, ref)


@pytest.mark.parametrize("seed", [1, 5, 11])
def test_fast_packed_records_equal_exact(seed, monkeypatch):
    """The key path knows each choice list's DP_FMT_P16D source while it makes
    the lists (a Dependency's first writer takes its row, a repeat names the
    first writer's list); the exact path derives them from the finished
    record (choice_sources).  Packed records are byte-for-byte equal, repeated
    and folded Dependencies included."""
    probs = _random_problems(seed, 400) + [
        [V("a", sat.Dependency("b", "c"), sat.Dependency("c"), sat.Dependency("b", "c")), V("b", sat.Dependency("c")),
         V("c")],
        [V("a", sat.Dependency("b", "b")), V("b")],
        [V("a", sat.Dependency("a")), V("b")],
        [V("a", sat.Dependency("b", "a")), V("b", sat.Dependency("a"), sat.Dependency("a"))]]
    wire = sat.encode_inputs(probs)
    fast = _lib.Lowered(wire, narrow=True, packed=True)
    monkeypatch.setenv("DEPPY_LOWER_EXACT", "1")
    exact = _lib.Lowered(wire, narrow=True, packed=True)
    assert exact.n_exact == len(probs) and fast.n_exact < 0.5 * len(probs)
    np.testing.assert_array_equal(fast.rec_off, exact.rec_off)
    np.testing.assert_array_equal(fast.rec, exact.rec)
    np.testing.assert_array_equal(fast.ident_var, exact.ident_var)
    np.testing.assert_array_equal(fast.ident_con, exact.ident_con)
    assert fast.msg == exact.msg
    fmts = np.array([int(fast.record(p)[13]) for p in range(fast.n)])
    assert np.isin(fmts, (5, 6)).sum() > 0.3 * fast.n


def test_relower_reuses_storage():
    a, b = _random_problems(7, 50), _random_problems(8, 80)
    lw = _lib.Lowered(sat.encode_inputs(a))
    keep = lw.rec.copy()
    fresh_b = _lib.Lowered(sat.encode_inputs(b))
    lw.relower(sat.encode_inputs(b))
    np.testing.assert_array_equal(lw.rec, fresh_b.rec)
    np.testing.assert_array_equal(lw.rec_off, fresh_b.rec_off)
    assert lw.msg == fresh_b.msg
    lw.relower(sat.encode_inputs(a))
    np.testing.assert_array_equal(lw.rec, keep)


@pytest.mark.parametrize("seed", [11, 12])
def test_packed_forms_of_colliding_problems(seed):
    """Random small problems with repeated and folded Dependencies, lowered
    in the packed forms: every DP_FMT_P16D / DP_FMT_P16 record widens back to
    its int32 record (dp_rec_widen and the independent restatement), and
    choice lists that repeat an earlier one (a Dependency whose gate an
    earlier one of the same subject emitted) are encoded as repeats."""
    from tests.gpu_common import unpack_p16, unpack_p8
    probs = _random_problems(seed, 400) + [
        [V("a", sat.Dependency("b", "c"), sat.Dependency("c"), sat.Dependency("b", "c")), V("b", sat.Dependency("c")),
         V("c")]]
    wire = sat.encode_inputs(probs)
    a = _lib.Lowered(wire)
    b = _lib.Lowered(wire, narrow=True, packed=True)
    L = _lib.lib()
    fmts = {}
    repeats = 0
    for p in range(a.n):
        r = np.ascontiguousarray(b.record(p))
        fmt = int(r[13])
        fmts[fmt] = fmts.get(fmt, 0) + 1
        out = np.zeros(int(r[10]), np.int32)
        assert L.dp_rec_widen(r.ctypes.data_as(_lib.c_i32p), len(r), out.ctypes.data_as(_lib.c_i32p)) == 0
        np.testing.assert_array_equal(out, a.record(p))
        if fmt in (3, 5, 6):
            np.testing.assert_array_equal(unpack_p16(r), a.record(p))
        if fmt == 6:
            r = unpack_p8(r)  # (its DP_FMT_P16D record)
        if fmt in (5, 6):
            nc, nk, nch, ncl, nkl, na = (int(r[i]) for i in (2, 3, 4, 7, 8, 5))
            tail = (2 * (ncl + nkl + nk + na) + 15) // 16 * 16
            repeats += int(np.count_nonzero(r[16:].view(np.uint8)[tail + nc + nk:tail + nc + nk + nch]))
    assert fmts.get(5, 0) + fmts.get(6, 0) > 0.3 * a.n, fmts
    assert repeats > 0


def test_packed_form_falls_back_when_rows_do_not_imply_lists():
    """DP_FMT_P16D only where the dependency rows give back the choice lists
    exactly: a Dependency whose gate folds away (Dependency(v; v) is always
    true: a choice list without a row) or whose candidates repeat (the Or
    chain drops the repeat: the row is shorter than the list) leaves the
    record in DP_FMT_P16 (or U16); every form widens to the same int32
    record."""
    from tests.gpu_common import unpack_p16
    cases = {
        "self": [V("a", sat.Dependency("a")), V("b")],
        "repeat": [V("a", sat.Dependency("b", "b")), V("b")],
        "plain": [V("a", sat.Dependency("b", "c")), V("b"), V("c")],
        "same-twice": [V("a", sat.Dependency("b"), sat.Dependency("b")), V("b")],
    }
    probs = list(cases.values())
    wire = sat.encode_inputs(probs)
    a = _lib.Lowered(wire)
    b = _lib.Lowered(wire, narrow=True, packed=True)
    L = _lib.lib()
    fmts = {}
    for p, name in enumerate(cases):
        r = np.ascontiguousarray(b.record(p))
        fmts[name] = int(r[13])
        out = np.zeros(int(r[10]), np.int32)
        assert L.dp_rec_widen(r.ctypes.data_as(_lib.c_i32p), len(r), out.ctypes.data_as(_lib.c_i32p)) == 0
        np.testing.assert_array_equal(out, a.record(p))
        if fmts[name] in (3, 5, 6):
            np.testing.assert_array_equal(unpack_p16(r), a.record(p))
    assert fmts["plain"] == 6 and fmts["same-twice"] == 6  # (DP_FMT_P8D: DP_FMT_P16D in 8 bits)
    assert fmts["self"] not in (5, 6) and fmts["repeat"] not in (5, 6), fmts


def test_bench_input_config_shape():
    """Config 6: problems of the reference's BenchmarkInput distribution
    (pkg/sat/bench_test.go:10-64) -- 256 variables "0".."255"; Mandatory with
    p=0.1, one Dependency of 1-5 other variables with p=0.15, 1-2 Conflicts
    with p=0.05, in that order -- lower and solve (oracle) without errors."""
    from oracle import oracle
    w = _lib.generate(6, 200, 9)
    pvo, vco, kind, cao = w["prob_var_off"], w["var_con_off"], w["con_kind"], w["con_arg_off"]
    assert np.all(np.diff(pvo) == 256)
    nv = int(pvo[-1])
    per = np.diff(vco)
    first = kind[vco[:-1][per > 0]]
    mand = (kind == 1).sum() / nv
    dep = kind == 3
    deps_per_var = np.diff(np.concatenate([[0], np.cumsum(dep)])[vco])
    assert 0.08 < mand < 0.12 and 0.13 < (deps_per_var > 0).mean() < 0.17 and deps_per_var.max() == 1
    nargs = np.diff(cao)[dep]
    assert nargs.min() == 1 and nargs.max() == 5
    conf_vars = np.diff(np.concatenate([[0], np.cumsum(kind == 4)])[vco])
    assert 0.035 < (conf_vars > 0).mean() < 0.065 and conf_vars.max() == 2
    assert set(np.unique(first)) <= {1, 3, 4}
    lw = _lib.Lowered(_lib.WireArrays(**{k: w[k] for k in (
        "prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off", "con_arg",
        "str_off")}, str_bytes=w["str_bytes"].tobytes()))
    assert (lw.err == 0).all()
    res = oracle.solve_batch(lw.rec_off, lw.rec, 0, 4)
    assert set(np.unique(res["status"])) <= {1, -1}
