"""Parity of the HIP path (libdeppy_hip.so on an MI355X) with the CPU
restatement (oracle/) and with the reference's own test vectors.

Run on the GPU box:  python -m pytest tests -m gpu
"""
import io
import sys

import numpy as np
import pytest

from deppy_amd import _lib, sat
from oracle import oracle
from tests import fixtures
from tests.gpu_common import compare_results, corrupt16, lowered_config
from tests.test_lowering import V, sat_var

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = _lib.Context(0, 1)
    yield c
    c.close()


def test_native_library_is_loaded(ctx):
    # the product path is the in-tree HIP library, nothing else
    maps = open("/proc/self/maps").read()
    assert _lib.LIB_PATH in maps


# ---------------------------------------------------------------------------
# the reference's own tests, through the full product path
# ---------------------------------------------------------------------------
SOLVE = fixtures.load("testsolve")["cases"] + fixtures.load("readme")["cases"]


@pytest.mark.parametrize("case", SOLVE, ids=[c["name"] for c in SOLVE])
def test_solve_golden(case):
    """pkg/sat/solve_test.go TestSolve, verbatim semantics (:299-355)."""
    variables = [sat_var(v) for v in case["variables"]]
    traces = io.StringIO()
    s, err = sat.NewSolver(sat.WithInput(variables), sat.WithTracer(sat.LoggingTracer(traces)))
    assert err is None
    installed, err = s.Solve(None)
    ids = sorted(str(v.Identifier()) for v in (installed or [])) or None
    assert ids == case["installed"]
    if case["error"] is None:
        assert err is None
    else:
        assert isinstance(err, sat.NotSatisfiable)
        got = sorted(err, key=lambda a: (str(a.Variable.Identifier()).encode(),
                                         a.Variable.Constraints().index(a.Constraint)))
        expect = []
        by = {str(v.Identifier()): v for v in variables}
        for a in case["error"]["applied"]:
            var = by[a["var"]]
            expect.append(sat.AppliedConstraint(var, var.Constraints()[a["constraint"]]))
        assert got == expect
        assert sat.NotSatisfiable(got).Error() == case["error"]["string"]


def test_duplicate_identifier():
    _, err = sat.NewSolver(sat.WithInput([V("a"), V("a")]))
    assert err == sat.DuplicateIdentifier("a")
    assert err.Error() == 'duplicate identifier "a" in input'


def test_lookup_error_surface():
    """An unknown identifier fails Solve with the aggregate error
    (lit_mapping.go:81-88, 119-128; solve.go:54-61).  The message format is
    pinned; the COUNT is parity-unpinned: the reference appends one error per
    lookup, at Apply time (counted here) and again in PushGuess for every
    Order() entry of each guessed variable (search.go:59-63), and whether its
    search runs at all depends on how gini propagates the z.LitNull operand
    the failed lookup leaves in the constraint's gate (not restatable without
    gini).  This build reports the Apply-time count, a lower
    bound of the reference's."""
    import re
    s, err = sat.NewSolver(sat.WithInput([V("a", sat.Mandatory(), sat.Dependency("x"))]))
    assert err is None
    installed, err = s.Solve(None)
    assert installed is None
    m = re.fullmatch(r'(\d+) errors encountered: variable "x" referenced but not provided'
                     r'(, variable "x" referenced but not provided)*', err.Error())
    assert m and int(m.group(1)) == err.Error().count("referenced but not provided") >= 1


def test_batch_mixed_with_errors():
    inputs = [[V("a", sat.Mandatory())], [V("a"), V("a")], [],
              [V("a", sat.Mandatory(), sat.Prohibited())]]
    out = sat.SolveBatch(inputs)
    assert [v.Identifier() for v in out[0][0]] == ["a"] and out[0][1] is None
    assert isinstance(out[1][1], sat.DuplicateIdentifier)
    assert out[2] == (None, None)
    assert isinstance(out[3][1], sat.NotSatisfiable) and len(out[3][1]) == 2


def test_golden_records_bit_exact(ctx):
    lw = _lib.Lowered(sat.encode_inputs([[sat_var(v) for v in c["variables"]] for c in SOLVE]))
    g = ctx.solve(lw.rec_off, lw.rec)
    o = oracle.solve_batch(lw.rec_off, lw.rec)
    assert compare_results(g, o, lw.n) == []


# ---------------------------------------------------------------------------
# seeded synthetic batches: bit-exact against the oracle
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("config,n,seed", [(2, 3000, 11), (3, 8000, 12), (5, 300, 13), (6, 3000, 14)])
def test_generated_bit_exact(ctx, config, n, seed):
    lw = lowered_config(config, n, seed)
    g = ctx.solve(lw.rec_off, lw.rec)
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    bad = compare_results(g, o, n)
    assert bad == [], bad[:10]
    st = g["status"]
    print("config", config, "SAT", int((st == 1).sum()), "UNSAT", int((st == -1).sum()),
          "INCOMPLETE", int((st == 0).sum()), "ERROR", int((st == -2).sum()),
          "class B", int(((g["flags"] & 2) != 0).sum()), file=sys.stderr)


@pytest.mark.parametrize("config,n,seed", [(4, 6, 31)])
def test_olm_scale_bit_exact(ctx, config, n, seed):
    """Config 4: OLM-scale catalogs (V~55k), one multi-wave workgroup each."""
    lw = lowered_config(config, n, seed)
    assert min(int(lw.record(p)[1]) for p in range(n)) > 50000
    g = ctx.solve(lw.rec_off, lw.rec)
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    bad = compare_results(g, o, n)
    assert bad == [], bad[:10]
    assert (g["status"] == 1).all()


@pytest.mark.parametrize("flags", [_lib.OPT_FORCE_GROUP, _lib.OPT_FORCE_MID, _lib.OPT_FORCE_HBM],
                         ids=["split", "split4", "hbm"])
@pytest.mark.parametrize("config,n,seed", [(2, 300, 41), (5, 120, 42), (3, 500, 43)])
def test_multiwave_paths_bit_exact(config, n, seed, flags):
    """The workgroup-per-problem kernels (M_SPLIT, M_SPLIT4, M_HBM) on small catalogs,
    where the oracle is cheap and every path (learning, epilogue, cores) is hit."""
    c = _lib.Context(0, 1, flags=flags)
    try:
        lw = lowered_config(config, n, seed)
        g = c.solve(lw.rec_off, lw.rec)
    finally:
        c.close()
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    bad = compare_results(g, o, n)
    assert bad == [], bad[:10]


@pytest.mark.parametrize("form", ["i32", "u16", "packed"])
@pytest.mark.parametrize("config,n,seed", [(2, 300, 141), (5, 150, 142), (3, 500, 143), (6, 300, 144)])
def test_ldsg_paths_bit_exact(config, n, seed, form):
    """The all-LDS multi-wave workgroup (M_LDSG, forced by DP_OPT_FORCE_LDSG)
    on small catalogs, where the oracle is cheap: int32 records narrowed and
    checked on the host, 16-bit records validated by the kernel, packed
    records decoded by one wavefront -- every field bit-exact."""
    lw = lowered_config(config, n, seed, narrow=form != "i32", packed=form == "packed")
    c = _lib.Context(0, 1, flags=_lib.OPT_FORCE_LDSG)
    try:
        g = c.solve(lw.rec_off, lw.rec)
    finally:
        c.close()
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    bad = compare_results(g, o, n)
    assert bad == [], bad[:10]


@pytest.mark.parametrize("flags", [_lib.OPT_FORCE_MID, _lib.OPT_FORCE_GROUP], ids=["split4", "split"])
@pytest.mark.parametrize("config,n,seed", [(2, 200, 44), (5, 80, 45)])
def test_round_table_overflow_bit_exact(config, n, seed, flags):
    """Multi-wave rounds whose implications overflow the LDS round table are
    redone on the HBM arrays (solve_kernel.hpp run_round); with 4-slot tables
    (DP_OPT_TINY_TABLE) nearly every round takes that path, and the trail
    ring wraps, so the frontier comes from HBM: results stay bit-exact."""
    c = _lib.Context(0, 1, flags=flags | _lib.OPT_TINY_TABLE)
    try:
        lw = lowered_config(config, n, seed)
        g = c.solve(lw.rec_off, lw.rec)
    finally:
        c.close()
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    bad = compare_results(g, o, n)
    assert bad == [], bad[:10]


@pytest.mark.parametrize("config,n,seed", [(2, 400, 21), (5, 60, 22)])
def test_models_and_cores_verified(ctx, config, n, seed):
    """Every SAT answer satisfies every row; every core is UNSAT on its own and
    deletion-minimal (north_star: 'a verified conflicting constraint subset')."""
    lw = lowered_config(config, n, seed)
    g = ctx.solve(lw.rec_off, lw.rec)
    for p in range(n):
        rec = lw.record(p)
        if g["status"][p] == 1:
            a0, a1 = g["inst_off"][p], g["inst_off"][p + 1]
            assert oracle.check_model(rec, g["installed"][a0:a1]) == -1
        elif g["status"][p] == -1 and not g["flags"][p] & 32:
            core = _lib.core_list(g, p)
            assert oracle.refute(rec, core) == -1
            for drop in core:
                assert oracle.refute(rec, [i for i in core if i != drop]) == 1


def test_full_size_properties(ctx):
    """BASELINE config 2 at full size (10k catalogs): deterministic, models
    check out, verdicts agree with the oracle on a sample."""
    lw = lowered_config(2, 10000, 2024)
    r = ctx.upload(lw.rec_off, lw.rec)
    try:
        r.run()
        a = r.download()
        r.run()
        b = r.download()
    finally:
        r.free()
    for k in ("status", "flags", "installed", "core", "core_len", "steps"):
        np.testing.assert_array_equal(a[k], b[k])
    assert (a["status"] != 0).all() and (a["status"] != -2).all()
    rng = np.random.default_rng(0)
    sample = rng.choice(10000, 500, replace=False)
    for p in sample:
        st, fl, inst, core, steps = oracle.solve(lw.record(p))
        assert st == a["status"][p] and fl == a["flags"][p]
        assert inst == _lib.installed_list(a, p, int(lw.record(p)[1]))
        assert core == _lib.core_list(a, p)


def test_empty_batch(ctx):
    g = ctx.solve(np.zeros(1, np.int64), np.zeros(0, np.int32))
    assert len(g["status"]) == 0


def test_pipelined_launches_match_serial(ctx):
    """dp_launch/dp_wait with several batches in flight on different streams
    give the same results as dp_run, and a relaunch waits for the previous one."""
    lw = lowered_config(5, 400, 31)
    lw2 = lowered_config(2, 600, 32)
    ref = ctx.solve(lw.rec_off, lw.rec)
    ref2 = ctx.solve(lw2.rec_off, lw2.rec)
    slots = [ctx.upload(lw.rec_off, lw.rec), ctx.upload(lw2.rec_off, lw2.rec), ctx.upload(lw.rec_off, lw.rec)]
    try:
        for _ in range(3):
            for s in slots:
                s.launch()
        slots[1].launch()  # still in flight: waits, then relaunches
        outs = [s.download() for s in slots]  # download waits
    finally:
        for s in slots:
            s.free()
    for out, want, n in ((outs[0], ref, 400), (outs[1], ref2, 600), (outs[2], ref, 400)):
        assert compare_results(out, want, n) == []


# ---------------------------------------------------------------------------
# the host-to-host pipeline (dp_submit / dp_job_wait) and the record forms
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("config,n,seed", [(2, 2000, 51), (3, 5000, 52), (5, 300, 53)])
def test_narrow_records_bit_exact(ctx, config, n, seed):
    """16-bit-form records (dp_lower_into DP_LOWER_NARROW) solve exactly like
    their int32 form, and like the oracle."""
    a = lowered_config(config, n, seed)
    b = lowered_config(config, n, seed, narrow=True)
    ga = ctx.solve(a.rec_off, a.rec)
    gb = ctx.solve(b.rec_off, b.rec)
    assert compare_results(gb, ga, n) == []
    o = oracle.solve_batch(b.rec_off, b.rec, 0, 16)
    assert compare_results(gb, o, n) == []


def test_jobs_in_flight_small_chunks(monkeypatch):
    """Many chunks per job and several jobs in flight: lanes are reused across
    jobs (a submit first delivers the lane's previous chunk), and every job's
    results equal its own synchronous solve."""
    monkeypatch.setenv("DEPPY_CHUNK_PROBLEMS", "97")
    c = _lib.Context(0, 1)
    try:
        batches = [lowered_config(cfg, n, s, narrow=s % 2 == 0)
                   for cfg, n, s in ((2, 700, 61), (5, 150, 62), (3, 2500, 63), (2, 300, 64))]
        refs = [oracle.solve_batch(b.rec_off, b.rec, 0, 16) for b in batches]
        jobs = [c.submit(b.rec_off, b.rec) for b in batches]
        outs = [j.wait() for j in jobs]
        st = c.stats()
        assert st["chunks"] >= sum(-(-b.n // 97) for b in batches)
    finally:
        c.close()
    for out, ref, b in zip(outs, refs, batches):
        assert compare_results(out, ref, b.n) == []


@pytest.mark.parametrize("flags", [0, _lib.OPT_FORCE_GROUP, _lib.OPT_FORCE_LDSG], ids=["lds", "group", "ldsg"])
def test_malformed_records_are_per_problem_errors(flags):
    """A malformed record yields DP_ERROR + DP_F_MALFORMED for that problem
    (found while narrowing on the host, or by the kernel's own validation)
    and the rest of the batch is solved bit-exactly."""
    lw = lowered_config(2, 40, 71)
    rec = lw.rec.copy()
    bad = [3, 17, 30]
    for p in bad:
        r0 = int(lw.rec_off[p])
        nc = int(rec[r0 + 2])
        if p == 3:
            rec[r0 + 16 + nc + 1] = 2 * int(rec[r0 + 1]) + 3   # clause literal past 2*nv
        elif p == 17:
            rec[r0 + 16 + 1] = rec[r0 + 16 + 2] + 1             # clause offsets decrease
        else:
            nk, ncl, nkl = int(rec[r0 + 3]), int(rec[r0 + 7]), int(rec[r0 + 8])
            cl = r0 + 16 + nc + 1 + ncl + nc + nk + 1           # card_lits
            rec[cl] = int(rec[r0 + 1]) + 7                      # AtMost variable past nv
    c = _lib.Context(0, 1, flags=flags)
    try:
        g = c.solve(lw.rec_off, rec)
    finally:
        c.close()
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    for p in bad:
        assert g["status"][p] == -2 and g["flags"][p] == 512 and g["core_len"][p] == 0, p
    ok = [p for p in range(lw.n) if p not in bad]
    assert compare_results(g, o, lw.n, only=ok) == []  # every field, installed sets and cores too


@pytest.mark.parametrize("config,n,seed", [(2, 3000, 81), (3, 9000, 82), (5, 400, 83)])
def test_pinned_records_copied_directly(config, n, seed, monkeypatch):
    """A DP_LOWER_NARROW | DP_LOWER_PINNED batch goes to the device by DMA
    from where it lies (no staging): every chunk of an all-16-bit batch is
    direct, and the results equal the staged path's and the oracle's."""
    monkeypatch.setenv("DEPPY_CHUNK_PROBLEMS", "700")
    lw = lowered_config(config, n, seed, narrow=True, pinned=True)
    assert lw.pinned and np.all(lw.rec_off % 4 == 0)
    c = _lib.Context(0, 1)
    try:
        g = c.submit(lw.rec_off, lw.rec).wait()
        st = c.stats(reset=True)
        assert st["chunks"] == -(-n // 700)
        if config != 5:  # every record on the one-wavefront path: no staging at all
            assert st["direct_chunks"] == st["chunks"]
        # (config 5: chunks whose multi-wave records are a small part of them
        # go direct, those records staged after the copied range)
        staged = c.submit(lw.rec_off, lw.rec.copy()).wait()  # pageable copy: staged
        assert c.stats()["direct_chunks"] == 0
    finally:
        c.close()
    assert compare_results(g, staged, n) == []
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    assert compare_results(g, o, n) == []


@pytest.mark.parametrize("flags", [0, _lib.OPT_FORCE_LDSG], ids=["lds", "ldsg"])
@pytest.mark.parametrize("pinned", [False, True], ids=["staged", "direct"])
def test_malformed_16bit_records_found_by_the_kernel(pinned, flags):
    """16-bit records the host passes through unread are validated by the
    kernel (Group::valid_record): each malformed one is DP_ERROR +
    DP_F_MALFORMED, the rest of the batch is solved bit-exactly."""
    lw = lowered_config(2, 60, 91, narrow=True, pinned=pinned)
    ref = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    rec = lw.rec if pinned else lw.rec.copy()
    bad = []
    for p, kind in ((4, "lit"), (19, "off"), (33, "run"), (47, "run")):
        if corrupt16(lw.rec_off, rec, p, kind):
            bad.append(p)
    assert len(bad) >= 3
    c = _lib.Context(0, 1, flags=flags)
    try:
        g = c.solve(lw.rec_off, rec)
        assert (c.stats()["direct_chunks"] > 0) == pinned
    finally:
        c.close()
    ok = [p for p in range(lw.n) if p not in bad]
    for p in bad:
        assert g["status"][p] == -2 and g["flags"][p] == 512 and g["core_len"][p] == 0, p
    assert compare_results(g, ref, lw.n, only=ok) == []


@pytest.mark.parametrize("config,n,seed,flags,p8", [(2, 3000, 101, 0, True), (3, 9000, 102, 0, True),
                                                    (5, 300, 103, 0, True), (6, 3000, 104, 0, True),
                                                    (2, 200, 104, _lib.OPT_FORCE_GROUP, True),
                                                    (2, 200, 105, _lib.OPT_FORCE_LDSG, True),
                                                    (2, 3000, 101, 0, False), (5, 300, 103, 0, False)],
                         ids=["c2", "c3", "c5", "c6", "c2-group", "c2-ldsg", "c2-p16d", "c5-p16d"])
def test_packed_records_bit_exact(config, n, seed, flags, p8):
    """Packed records (dp_lower_into DP_LOWER_PACKED: DP_FMT_P8D up to 512
    variables, else DP_FMT_P16D; p8=False: DP_FMT_P16D), copied to the device
    as they lie and decoded by the kernel (or widened on the host for a
    multi-wave placement), solve exactly like their int32 form and the oracle."""
    a = lowered_config(config, n, seed)
    b = lowered_config(config, n, seed, packed=True, pinned=True, p8=p8)
    fmts = set(b.rec[b.rec_off[:-1] + 13].tolist())
    assert (6 in fmts) == (p8 and config != 4), fmts
    c = _lib.Context(0, 1, flags=flags)
    try:
        gb = c.submit(b.rec_off, b.rec).wait()
        direct = c.stats()["direct_chunks"]
        ga = c.solve(a.rec_off, a.rec)
    finally:
        c.close()
    if flags == 0 and config != 5:
        assert direct > 0
    assert compare_results(gb, ga, n) == []
    o = oracle.solve_batch(a.rec_off, a.rec, 0, 16)
    assert compare_results(gb, o, n) == []


@pytest.mark.parametrize("flags", [0, _lib.OPT_FORCE_LDSG], ids=["lds", "ldsg"])
def test_malformed_packed_records_found_by_the_kernel(flags):
    """Packed records are validated on the device: a wrong identity mask, row
    lengths that do not sum to the total, an out-of-range literal, dependency
    rows that no longer imply the header's choice lists (DP_FMT_P16D) ->
    DP_ERROR + DP_F_MALFORMED for that problem only."""
    lw = lowered_config(2, 40, 111, packed=True, pinned=True, p8=False)
    ref = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    rec = lw.rec
    bad = [5, 12, 27, 33]
    for p, kind in zip(bad, ("mask", "len", "lit", "dep")):
        r = rec[lw.rec_off[p]:lw.rec_off[p + 1]]
        assert r[13] == 5
        nv, nc, nk, nch, na, nid, ncl, nkl, nchl = (int(r[i]) for i in range(1, 10))
        tail = (2 * (ncl + nkl + nk + na) + 15) // 16 * 16
        t = r[16:].view(np.uint8)
        u = r[16:].view(np.uint16)
        if kind == "mask":
            t[tail + nc + nk + nch] ^= 1
        elif kind == "len":
            t[tail] += 1
        elif kind == "lit":
            u[0] = 2 * nv + 1
        else:  # a dependency row's first literal made positive: one list short
            offs = np.concatenate([[0], np.cumsum(t[tail:tail + nc].astype(np.int64))])
            a = next(a for a, e in zip(offs[:-1], offs[1:]) if e - a >= 2 and u[a] & 1 and not np.any(u[a + 1:e] & 1))
            u[a] ^= 1
    c = _lib.Context(0, 1, flags=flags)
    try:
        g = c.solve(lw.rec_off, rec)
    finally:
        c.close()
    ok = [p for p in range(lw.n) if p not in bad]
    for p in bad:
        assert g["status"][p] == -2 and g["flags"][p] == 512 and g["core_len"][p] == 0, p
    assert compare_results(g, ref, lw.n, only=ok) == []


@pytest.mark.parametrize("flags", [0, _lib.OPT_FORCE_LDSG], ids=["lds", "ldsg"])
def test_malformed_p8_records_found_by_the_kernel(flags):
    """DP_FMT_P8D records are decoded and validated on the device: an unknown
    flag bit, a list source marked nonzero that is zero, a variable past nv,
    row lengths that do not sum to the total -> DP_ERROR + DP_F_MALFORMED for
    that problem only, the others bit-exact."""
    from tests.gpu_common import p8_sections
    lw = lowered_config(2, 60, 112, packed=True, pinned=True)
    ref = oracle.solve_batch(lw.rec_off, lw.rec, 0, 16)
    rec = lw.rec
    cand = [p for p in range(lw.n) if int(rec[lw.rec_off[p] + 1]) < 256 and rec[lw.rec_off[p] + 14] & 4
            and p8_sections(rec[lw.rec_off[p]:lw.rec_off[p + 1]])["nz"] > 0]
    bad = cand[:4]
    assert len(bad) == 4
    for p, kind in zip(bad, ("flag", "src", "var", "len")):
        r = rec[lw.rec_off[p]:lw.rec_off[p + 1]]
        assert r[13] == 6
        S = p8_sections(r)
        t = r[16:].view(np.uint8)
        if kind == "flag":
            r[14] |= 64
        elif kind == "src":
            t[S["srcval"]] = 0
        elif kind == "var":
            t[0] = 255
        else:
            t[S["lens"]] ^= 1
    c = _lib.Context(0, 1, flags=flags)
    try:
        g = c.solve(lw.rec_off, rec)
    finally:
        c.close()
    ok = [p for p in range(lw.n) if p not in bad]
    for p in bad:
        assert g["status"][p] == -2 and g["flags"][p] == 512 and g["core_len"][p] == 0, p
    assert compare_results(g, ref, lw.n, only=ok) == []


def test_p8_wide_variables_bit_exact():
    """DP_FMT_P8D with the bit-8 planes (257..512 variables), byte bounds and
    byte lengths, beside DP_FMT_P16D past 512 variables: decoded on the
    device, bit-exact with the int32 records and the oracle."""
    from tests.gpu_common import wide_problems
    wire = sat.encode_inputs(wide_problems(7, 24, [300, 512, 513, 200, 450]))
    a = _lib.Lowered(wire)
    b = _lib.Lowered(wire, narrow=True, packed=True, pinned=True)
    fmts = b.rec[b.rec_off[:-1] + 13]
    assert (fmts == 6).sum() >= 16 and (fmts == 5).sum() >= 4, fmts
    c = _lib.Context(0, 1)
    try:
        g = c.submit(b.rec_off, b.rec).wait()
    finally:
        c.close()
    assert compare_results(g, oracle.solve_batch(a.rec_off, a.rec, 0, 16), a.n) == []


def test_packed_tail_larger_than_watch_room_bit_exact():
    """The kernel copies a packed record's tail past the decoded arrays (where
    the watch lists go later) while it decodes it; layout() grows the body
    when the tail is larger than that room: few variables with many repeated
    Dependencies (DP_FMT_P16D with 200 repeats; DP_FMT_P16 with 200 repeats of
    a Dependency that names its candidate twice, whose row is shorter than its
    list), beside an ordinary catalog."""
    probs = [[V("a", *[sat.Dependency("b") for _ in range(200)]), V("b", sat.Mandatory())],
             [V("x", sat.Mandatory(), *[sat.Dependency("y", "y") for _ in range(200)]), V("y")],
             [V("p", sat.Mandatory(), sat.Dependency("q")), V("q", sat.Prohibited())]]
    wire = sat.encode_inputs(probs)
    a = _lib.Lowered(wire)
    b = _lib.Lowered(wire, narrow=True, packed=True, pinned=True)
    fmts = [int(b.record(p)[13]) for p in range(b.n)]
    assert fmts[0] == 6 and fmts[1] == 3, fmts  # (DP_FMT_P8D: its tail expanded after its bytes)
    for p in range(b.n):  # the tail is larger than the record's watch-list room
        h = b.record(p)
        nv, nc, nk, nch, nid, ncl, nkl = (int(h[i]) for i in (1, 2, 3, 4, 6, 7, 8))
        tb = nc + nk + nch + (nid + 7) // 8 + (nv if fmts[p] == 3 else 0)
        if p < 2:
            assert tb > 2 * (2 * nv + 1 + ncl + nkl), (p, tb)
    c = _lib.Context(0, 1)
    try:
        g = c.submit(b.rec_off, b.rec).wait()
    finally:
        c.close()
    assert compare_results(g, oracle.solve_batch(a.rec_off, a.rec, 0, 16), a.n) == []
    assert list(g["status"]) == [1, 1, -1]


def test_explicit_choice_packed_records_bit_exact():
    """DP_FMT_P16 records (explicit choice lists, as a producer that does not
    derive them packs them) are decoded by the kernel like DP_FMT_P16D."""
    from tests.gpu_common import pack_p16
    a = lowered_config(2, 500, 131)
    parts = [pack_p16(a.record(p)) for p in range(a.n)]
    off = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.int64)
    rec = np.concatenate(parts).astype(np.int32)
    assert np.all(rec[off[:-1] + 13] == 3)
    c = _lib.Context(0, 1)
    try:
        g = c.solve(off, rec)
    finally:
        c.close()
    assert compare_results(g, oracle.solve_batch(a.rec_off, a.rec, 0, 16), a.n) == []


def test_wide_records_direct_and_validated(monkeypatch):
    """Multi-wave records in the DP_FMT_I32W form (record + watch lists, as
    dp_lower_into emits them under DEPPY_HOST_WATCHES=1) go to the device as
    they lie; the kernel checks their bounds: a watch entry past the rows, a
    clause literal past 2nv -> DP_F_MALFORMED for that problem, the rest
    exact."""
    a = lowered_config(5, 120, 121)
    monkeypatch.setenv("DEPPY_HOST_WATCHES", "1")
    monkeypatch.setenv("DEPPY_LDSG", "0")  # mid-size catalogs as HBM-read multi-wave records
    b = lowered_config(5, 120, 121, packed=True, pinned=True)
    wide = [p for p in range(b.n) if b.rec[b.rec_off[p] + 13] == 4]
    assert len(wide) >= 3
    ref = oracle.solve_batch(a.rec_off, a.rec, 0, 16)
    c = _lib.Context(0, 1)
    try:
        g = c.submit(b.rec_off, b.rec).wait()
        assert c.stats(reset=True)["direct_chunks"] > 0
        assert compare_results(g, ref, b.n) == []
        bad = wide[:2]
        r0 = b.rec[b.rec_off[bad[0]]:b.rec_off[bad[0] + 1]]
        words, nv = int(r0[10]), int(r0[1])
        r0[words + 2 * nv + 1] = int(r0[2]) + int(r0[3]) + 5      # first watch entry past the rows
        r1 = b.rec[b.rec_off[bad[1]]:b.rec_off[bad[1] + 1]]
        r1[16 + int(r1[2]) + 1] = 2 * int(r1[1]) + 1                # first clause literal past 2nv
        g = c.submit(b.rec_off, b.rec).wait()
    finally:
        c.close()
    ok = [p for p in range(b.n) if p not in bad]
    for p in bad:
        assert g["status"][p] == -2 and g["flags"][p] == 512, p
    assert compare_results(g, ref, b.n, only=ok) == []


def test_olm_scale_direct_bit_exact(ctx, monkeypatch):
    """OLM-scale catalogs (config 4) lowered to DP_FMT_I32W (host-built watch
    lists, DEPPY_HOST_WATCHES=1) and copied directly: the same result as
    their int32 form, whose lists the device builds, and the oracle."""
    a = lowered_config(4, 2, 131)
    monkeypatch.setenv("DEPPY_HOST_WATCHES", "1")
    b = lowered_config(4, 2, 131, narrow=True, pinned=True)
    assert np.all(b.rec[b.rec_off[:-1] + 13] == 4)
    gb = ctx.submit(b.rec_off, b.rec).wait()
    ga = ctx.solve(a.rec_off, a.rec)
    assert compare_results(gb, ga, 2) == []
    o = oracle.solve_batch(a.rec_off, a.rec, 0, 2)
    assert compare_results(gb, o, 2) == []


# ---------------------------------------------------------------------------
# round 3: queued grids at OLM scale, full-size config 5, plain int32
# multi-wave records, the device-watch-list boundary
# ---------------------------------------------------------------------------
def test_olm_scale_queued_grid_bit_exact(monkeypatch):
    """Config 4 through the persistent (queued) multi-wave grid with fewer
    workgroups than catalogs (DEPPY_GRID_CAP=4): every workgroup solves
    several catalogs in turn, re-initialising its LDS and scratch between
    them (solve_kernel.hpp solve_kernel's queue loop).  Bit-exact with the
    oracle, catalog by catalog."""
    monkeypatch.setenv("DEPPY_GRID_CAP", "4")
    n = 24
    a = lowered_config(4, n, 171)
    b = lowered_config(4, n, 171, narrow=True, pinned=True)
    c = _lib.Context(0, 1)
    try:
        gb = c.submit(b.rec_off, b.rec).wait()
        ga = c.solve(a.rec_off, a.rec)
    finally:
        c.close()
    o = oracle.solve_batch(a.rec_off, a.rec, 0, 16)
    assert compare_results(ga, o, n) == []
    assert compare_results(gb, o, n) == []


def test_olm_scale_many_catalogs_bit_exact(ctx):
    """More config-4 catalogs than one launch holds resident (the default
    queued grid): later catalogs are taken by workgroups that already
    finished one."""
    n = 600
    a = lowered_config(4, n, 181, narrow=True, pinned=True)
    g = ctx.submit(a.rec_off, a.rec).wait()
    w = lowered_config(4, n, 181)
    o = oracle.solve_batch(w.rec_off, w.rec, 0, 16)
    assert compare_results(g, o, n) == []


def test_config5_full_size_bit_exact(ctx):
    """BASELINE config 5 at its bench size (10k mixed-size catalogs, half of
    them with an injected infeasibility): every field of every catalog, cores
    included, equals the oracle's."""
    n = 10000
    lw = lowered_config(5, n, 2025, packed=True, pinned=True)
    g = ctx.submit(lw.rec_off, lw.rec).wait()
    w = lowered_config(5, n, 2025)
    o = oracle.solve_batch(w.rec_off, w.rec, 0, 16)
    bad = compare_results(g, o, n)
    assert bad == [], bad[:10]
    assert (g["status"] == -1).sum() > n // 4


def test_plain_int32_multiwave_records_validated_by_the_kernel(monkeypatch):
    """Multi-wave records of at most 2048 variables go to the device as plain
    int32 records (DP_FMT_I32) copied as they lie; the kernel checks them
    (valid_wide) before building their watch lists.  A clause literal past
    2nv, decreasing clause offsets and an AtMost variable past nv each give
    DP_ERROR + DP_F_MALFORMED for that problem only; the rest stay exact."""
    monkeypatch.setenv("DEPPY_LDSG", "0")  # mid-size catalogs as HBM-read multi-wave records
    a = lowered_config(5, 160, 191)
    b = lowered_config(5, 160, 191, packed=True, pinned=True)
    plain = [p for p in range(b.n) if b.rec[b.rec_off[p] + 13] == 0]
    assert len(plain) >= 3
    ref = oracle.solve_batch(a.rec_off, a.rec, 0, 16)
    bad = plain[:3]
    for p, kind in zip(bad, ("lit", "off", "card")):
        r = b.rec[b.rec_off[p]:b.rec_off[p + 1]]
        nv, nc, nk, ncl = int(r[1]), int(r[2]), int(r[3]), int(r[7])
        if kind == "lit":
            r[16 + nc + 1] = 2 * nv + 1
        elif kind == "off":
            r[16 + 1] = r[16 + 2] + 1
        else:
            assert nk > 0
            r[16 + nc + 1 + ncl + nc + nk + 1] = nv + 3
    c = _lib.Context(0, 1)
    try:
        g = c.submit(b.rec_off, b.rec).wait()
        assert c.stats()["direct_chunks"] > 0
    finally:
        c.close()
    for p in bad:
        assert g["status"][p] == -2 and g["flags"][p] == 512 and g["core_len"][p] == 0, p
    ok = [p for p in range(b.n) if p not in bad]
    assert compare_results(g, ref, b.n, only=ok) == []


def chain_catalog(n_vars, seed):
    """A catalog of exactly n_vars variables (layout.hpp DEV_WATCH_VARS
    boundary tests): packages of 9 versions newest first, each version
    depending on a version range of a later package, one uniqueness AtMost
    per package, and required variables for the rest of the count."""
    rng = np.random.default_rng(seed)
    n_pkg = (n_vars - 8) // 10
    req = n_vars - 10 * n_pkg
    names = [["p%d-v%d" % (p, 8 - i) for i in range(9)] for p in range(n_pkg)]
    out = []
    for p in range(n_pkg):
        for i in range(9):
            cons = []
            if p + 1 < n_pkg and rng.random() < 0.5:
                q = int(rng.integers(p + 1, min(n_pkg, p + 4)))
                lo = int(rng.integers(0, 9))
                cons.append(sat.Dependency(*names[q][lo:min(9, lo + int(rng.integers(1, 4)))]))
            if rng.random() < 0.05 and p > 0:
                cons.append(sat.Conflict(names[int(rng.integers(0, p))][int(rng.integers(0, 9))]))
            out.append(V(names[p][i], *cons))
        out.append(V("u%d" % p, sat.AtMost(1, *names[p])))
    for r in range(req):
        p = int(rng.integers(0, n_pkg))
        out.append(V("req%d" % r, sat.Mandatory(), sat.Dependency(*names[p])))
    assert len(out) == n_vars
    return out


@pytest.mark.parametrize("flags", [_lib.OPT_FORCE_GROUP, _lib.OPT_FORCE_MID, _lib.OPT_FORCE_HBM],
                         ids=["split", "split4", "hbm"])
def test_device_watch_boundary_bit_exact(flags, monkeypatch):
    """Catalogs of 2047, 2048 and 2049 variables on the multi-wave paths:
    up to 2048 the solving workgroup builds the watch lists (2nv+1 counters
    in the LDS work area), above it the grid-wide passes before the launch
    do (watch_build.hip).  Bit-exact with the oracle on both sides of the
    boundary."""
    monkeypatch.setenv("DEPPY_LDSG", "0")  # (else these fit the all-LDS group, as 16-bit records)
    probs = [chain_catalog(nv, 7 + nv) for nv in (2047, 2048, 2049)]
    # page-locked plain int32 records on 16-byte boundaries, as dp_lower_into
    # emits multi-wave records: dp_submit copies them as they lie, so the
    # device builds every list (a staged record would bring host-built ones)
    lw = _lib.Lowered(sat.encode_inputs(probs), narrow=True, packed=True, pinned=True)
    assert [int(lw.record(p)[1]) for p in range(3)] == [2047, 2048, 2049]
    assert [int(lw.record(p)[13]) for p in range(3)] == [0, 0, 0]  # DP_FMT_I32
    c = _lib.Context(0, 1, flags=flags)
    try:
        g = c.submit(lw.rec_off, lw.rec).wait()
        assert c.stats(reset=True)["direct_chunks"] > 0
    finally:
        c.close()
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 3)
    assert compare_results(g, o, 3) == []
    assert (g["status"] != -2).all()


def test_olm_scale_device_lists_bit_exact():
    """Config 4 as dp_lower_into emits it (plain int32, no watch lists): the
    records go to the device as they lie and the grid-wide passes build every
    catalog's lists before the launch (watch_build.hip).  Bit-exact with the
    oracle, catalog by catalog."""
    n = 12
    a = lowered_config(4, n, 181)
    b = lowered_config(4, n, 181, packed=True, pinned=True)
    assert np.all(b.rec[b.rec_off[:-1] + 13] == 0)
    c = _lib.Context(0, 1)
    try:
        g = c.submit(b.rec_off, b.rec).wait()
        assert c.stats(reset=True)["direct_chunks"] > 0
    finally:
        c.close()
    assert compare_results(g, oracle.solve_batch(a.rec_off, a.rec, 0, 16), n) == []


def test_olm_scale_device_lists_malformed():
    """The list passes run before the kernel validates a record: a clause
    literal past 2nv, and clause offsets out of range, in two OLM-scale
    records -> DP_F_MALFORMED for those two (their lists stay in bounds),
    every other catalog exact."""
    n = 6
    a = lowered_config(4, n, 191)
    b = lowered_config(4, n, 191, packed=True, pinned=True)
    ref = oracle.solve_batch(a.rec_off, a.rec, 0, 16)
    r1 = b.rec[b.rec_off[1]:b.rec_off[2]]
    nc1, nv1 = int(r1[2]), int(r1[1])
    r1[16 + nc1 + 1 + 7] = 2 * nv1 + 1            # a clause literal past 2nv
    r3 = b.rec[b.rec_off[3]:b.rec_off[4]]
    r3[16 + 5] = int(r3[7]) + 1000                # clause_off[5] past ncl
    c = _lib.Context(0, 1)
    try:
        g = c.submit(b.rec_off, b.rec).wait()
    finally:
        c.close()
    for p in (1, 3):
        assert g["status"][p] == -2 and g["flags"][p] == 512, p
    assert compare_results(g, ref, n, only=[0, 2, 4, 5]) == []


def long_row_catalog(n_vars, width, seed):
    """chain_catalog plus rows too long for a watch entry's packed range
    (layout.hpp row_info: 255 positions or more): one required variable
    depending on `width` candidates (a clause row of width + 1 literals) and
    an AtMost(1) over the same candidates (an AtMost row of `width`)."""
    base = chain_catalog(n_vars - 2, seed)
    cands = [str(v.Identifier()) for v in base[:width]]
    return base + [V("wide-req", sat.Mandatory(), sat.Dependency(*cands)),
                   V("wide-uniq", sat.AtMost(1, *cands))]


@pytest.mark.parametrize("n_vars", [600, 2400], ids=["in_kernel_lists", "device_passes"])
@pytest.mark.parametrize("flags", [_lib.OPT_FORCE_GROUP, _lib.OPT_FORCE_MID], ids=["split", "split4"])
def test_multiwave_long_rows_bit_exact(n_vars, flags):
    """Multi-wave watch entries carry their row's literal range, except rows
    of 255 or more positions, which keep ROW_INFO_NONE and are read through
    their offsets (clause rows in a visit and Solve()'s scan, AtMost rows in
    the flush).  Catalogs with a 300-literal dependency row and a 299-wide
    AtMost row, with lists built by the solving workgroup (600 variables)
    and by the grid-wide passes (2400): bit-exact with the oracle."""
    probs = [long_row_catalog(n_vars, 299, 11 + k) for k in range(3)]
    # plain int32 records, page-locked: copied as they lie, lists built on the device
    lw = _lib.Lowered(sat.encode_inputs(probs), pinned=True)
    assert [int(lw.record(p)[13]) for p in range(3)] == [0, 0, 0]  # DP_FMT_I32
    c = _lib.Context(0, 1, flags=flags)
    try:
        g = c.submit(lw.rec_off, lw.rec).wait()
        assert c.stats(reset=True)["direct_chunks"] > 0
    finally:
        c.close()
    o = oracle.solve_batch(lw.rec_off, lw.rec, 0, 3)
    assert compare_results(g, o, 3) == []
    assert (g["status"] != -2).all()


@pytest.mark.parametrize("config,n,seed", [(2, 3000, 151), (5, 300, 152)])
def test_multi_device_dispatcher_bit_exact(config, n, seed):
    """The one-process multi-device topology the cgo shim ships
    (dp_create(n_devices=2)): with DP_OPT_SHARE_ORDINAL both
    logical devices run on GPU 0, so the chunk cut, the per-device submitting
    threads and host pools, dp_partition of a resident batch and the result
    stitching run on hardware.  Both devices run chunks, and every field is
    bit-exact against the oracle on both the host-to-host and the resident
    path (reference caller: pkg/solver/solver.go:42-47)."""
    lw = lowered_config(config, n, seed, packed=True, pinned=True)
    w = lowered_config(config, n, seed)
    o = oracle.solve_batch(w.rec_off, w.rec, 0, 16)
    c = _lib.Context(0, 2, flags=_lib.OPT_SHARE_ORDINAL)
    try:
        assert c.devices() == 2
        c.stats(reset=True)
        g = c.submit(lw.rec_off, lw.rec).wait()
        per = [c.device_stats(d)["chunks"] for d in range(2)]
        assert min(per) >= 1, per
        assert sum(per) == c.stats()["chunks"]
        r = c.upload(lw.rec_off, lw.rec)
        try:
            r.run()
            gr = r.download()
        finally:
            r.free()
    finally:
        c.close()
    assert compare_results(g, o, n) == []
    assert compare_results(gr, o, n) == []


def test_multi_device_shared_queue_bit_exact(monkeypatch):
    """Several devices pull a job's chunks from the context's shared queue,
    costliest (most record words) first, whenever a device has a free lane
    (runtime.cpp take_shared): config 5's mixed sizes cut into six chunks
    over two logical devices on GPU 0.  Every chunk runs exactly once, both
    devices run some, the per-device kernel time is reported, and every field
    is bit-exact against the oracle (reference caller:
    pkg/solver/solver.go:42-47)."""
    monkeypatch.setenv("DEPPY_MIN_SHARED_CHUNK", "32")
    n = 600
    lw = lowered_config(5, n, 153, packed=True, pinned=True)
    w = lowered_config(5, n, 153)
    o = oracle.solve_batch(w.rec_off, w.rec, 0, 16)
    c = _lib.Context(0, 2, flags=_lib.OPT_SHARE_ORDINAL)
    try:
        c.stats(reset=True)
        g = c.submit(lw.rec_off, lw.rec).wait()
        per = [c.device_stats(d) for d in range(2)]
        tot = c.stats()
    finally:
        c.close()
    assert tot["chunks"] == 6 and sum(d["chunks"] for d in per) == 6, (tot["chunks"], per)
    assert min(d["chunks"] for d in per) >= 1
    assert sum(d["problems"] for d in per) == n
    assert all(d["kernel_ms"] > 0 for d in per)
    assert compare_results(g, o, n) == []


def test_pipelined_solve_wire_bit_exact(ctx, monkeypatch):
    """sat.solve_wire on a batch of more than 2 x SUB_BATCH catalogs (the
    SolveBatch path) lowers and solves it in overlapping sub-batches; every
    field equals one solve of the whole batch's packed records, and the
    stitched identities equal the whole lowering's."""
    from deppy_amd import sat
    monkeypatch.setattr(sat, "SUB_BATCH", 4096)
    n = 2 * sat.SUB_BATCH + 1234
    w = _lib.generate(5, n, 171)
    wa = _lib.WireArrays(**{k: w[k] for k in ("prob_var_off", "var_id", "var_con_off", "con_kind", "con_n",
                                              "con_arg_off", "con_arg", "str_off")}, str_bytes=w["str_bytes"].tobytes())
    lw, res = sat.solve_wire(wa, ctx)
    assert isinstance(lw, sat._Stitched) and lw.n == n
    whole = _lib.Lowered(wa, narrow=True, packed=True, pinned=True)
    g = ctx.solve(whole.rec_off, whole.rec)
    assert compare_results(res, g, n) == []
    for k in ("ident_off", "ident_var", "ident_con", "err"):
        np.testing.assert_array_equal(getattr(lw, k), getattr(whole, k))
