"""Lowering on the device (dp_lower_device, deppy_amd/csrc/lower_device.hip):
the compact 32-bit wire lowered by one wavefront per problem gives the same
dp_lowered as dp_lower_into(NARROW | PACKED) on the host, byte for byte --
records, offsets, identity owners (the reported AppliedConstraint,
lit_mapping.go:69-72), errors and their texts -- with the problems the kernel
does not take lowered on the host and spliced in."""
import ctypes

import numpy as np
import pytest

from deppy_amd import _lib, sat
from tests import fixtures
from tests.test_lowering import EDGE, V, _random_problems, all_golden_variable_sets, variables_of


def wire_of(config, n, seed):
    w = _lib.generate(config, n, seed)
    return _lib.WireArrays(**{k: w[k] for k in (
        "prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off", "con_arg",
        "str_off")}, str_bytes=w["str_bytes"].tobytes())


def assert_same(dev, host):
    assert dev.n == host.n
    np.testing.assert_array_equal(dev.rec_off, host.rec_off)
    np.testing.assert_array_equal(dev.rec, host.rec)
    np.testing.assert_array_equal(dev.ident_off, host.ident_off)
    np.testing.assert_array_equal(dev.ident_var, host.ident_var)
    np.testing.assert_array_equal(dev.ident_con, host.ident_con)
    np.testing.assert_array_equal(dev.err, host.err)
    assert dev.msg == host.msg


def test_wire32_arrays_without_device():
    """The compact wire holds the 64-bit wire's content (numpy memory when
    no device gives page-locked memory) and refuses what does not fit."""
    w = wire_of(2, 30, 5)
    w32 = _lib.Wire32Arrays(w, ids16=False)
    a, b = w32.a, w.a
    np.testing.assert_array_equal(a["prob_var_off"], b["prob_var_off"])
    np.testing.assert_array_equal(a["prob_con_off"], b["var_con_off"][b["prob_var_off"]])
    np.testing.assert_array_equal(a["prob_arg_off"], b["con_arg_off"][a["prob_con_off"]])
    np.testing.assert_array_equal(a["var_id"], b["var_id"])
    np.testing.assert_array_equal(np.concatenate([[0], np.cumsum(a["var_ncon"])]), b["var_con_off"])
    np.testing.assert_array_equal(np.concatenate([[0], np.cumsum(a["con_nargs"])]), b["con_arg_off"])
    np.testing.assert_array_equal(a["con_kn"] & 7, b["con_kind"])
    np.testing.assert_array_equal(a["con_kn"] >> 3, b["con_n"])
    np.testing.assert_array_equal(a["con_arg"], b["con_arg"])
    assert w32.nbytes() < 0.5 * sum(b[k].nbytes for k in ("prob_var_off", "var_id", "var_con_off", "con_kind",
                                                           "con_n", "con_arg_off", "con_arg"))
    s = w32.struct()
    assert s.n_problems == 30 and s.n_strs == len(b["str_off"]) - 1 and not s.var_id16
    # 16-bit string indices where the table allows them
    w16 = _lib.Wire32Arrays(w)
    assert w16.ids16 and "var_id" not in w16.a and w16.a["con_arg16"].dtype == np.uint16
    np.testing.assert_array_equal(w16.a["var_id16"], b["var_id"])
    np.testing.assert_array_equal(w16.a["con_arg16"], b["con_arg"])
    assert w16.nbytes() < 0.75 * w32.nbytes()
    s16 = w16.struct()
    assert s16.var_id16 and s16.con_arg16 and not s16.var_id and not s16.con_arg
    big = _lib.WireArrays(**{k: v.copy() for k, v in b.items() if k != "str_bytes"},
                          str_bytes=b["str_bytes"][:-1].tobytes())
    big.a["con_arg"][0] = 1 << 40
    with pytest.raises(ValueError, match="32 bits"):
        _lib.Wire32Arrays(big, ids16=False)
    with pytest.raises(ValueError, match="16 bits"):
        _lib.Wire32Arrays(big)
    e = _lib.Lowered.empty()
    assert e.n == 0 and list(e.rec_off) == [0] and e._flags == 1 | 2 | 4


@pytest.fixture(scope="module")
def dl():
    ctx = _lib.Context(0, 1)
    d = _lib.DeviceLowerer(ctx)
    yield d
    d.close()
    ctx.close()


def lower_both(dl, wire, ids16=True, **kw):
    host = _lib.Lowered(wire, narrow=True, pinned=True, packed=True, **kw)
    dev = dl.lower(_lib.Wire32Arrays(wire, ids16=ids16), _lib.Lowered.empty(pinned=True, **kw))
    return dev, host


@pytest.mark.gpu
@pytest.mark.parametrize("config,n,ids16", [(2, 10000, True), (2, 3000, False), (3, 20000, True), (6, 5000, True),
                                            (5, 300, True)])
def test_device_records_equal_host(dl, config, n, ids16):
    """Configs 2, 3 and 6 lower entirely on the device (config 6's
    Dependencies on their own subject give DP_FMT_P16 records: choice lists
    without rows); config 5's multi-wave catalogs go to the host; every byte
    equals dp_lower_into's, with 16- and 32-bit string indices."""
    dev, host = lower_both(dl, wire_of(config, n, 77), ids16=ids16)
    assert_same(dev, host)
    forms = np.unique(dev.rec[dev.rec_off[:-1] + 13], return_counts=True)
    print("config", config, "host-lowered", dl.host_count, "of", n, "forms", forms)
    if config in (2, 3, 6):
        assert dl.host_count == 0


@pytest.mark.gpu
def test_device_records_of_colliding_problems(dl):
    """Small random problems where identity keys collide (Conflict vs
    AtMost(1;a,b), repeated Dependencies, AtMosts over one set in two orders,
    multiplicities, tautologies, lookup errors) -- the kernel takes what its
    keys decide and the host the rest; the result equals the host's."""
    probs = []
    for seed in (1, 2, 3, 5, 11):
        probs += _random_problems(seed, 400)
    probs += EDGE + [variables_of(vs) for vs in all_golden_variable_sets()]
    probs += [
        [V("a", sat.Dependency("b", "c"), sat.Dependency("c"), sat.Dependency("b", "c")), V("b", sat.Dependency("c")),
         V("c")],
        [V("a", sat.Conflict("b"), sat.AtMost(1, "b", "a")), V("b", sat.AtMost(1, "a", "b"), sat.Conflict("a"))],
        [V("a", sat.AtMost(1, "a", "b", "c"), sat.AtMost(1, "a", "b", "c"), sat.AtMost(2, "c", "b", "a")), V("b"),
         V("c", sat.AtMost(0, "a", "b"), sat.AtMost(0, "b", "a"))],
    ]
    wire = sat.encode_inputs(probs)
    dev, host = lower_both(dl, wire)
    assert_same(dev, host)
    # both paths were exercised
    assert 0 < dl.host_count < len(probs), dl.host_count


@pytest.mark.gpu
def test_device_lowering_other_flags_and_reuse(dl):
    """Flags the kernel does not emit (P16D kept by DP_LOWER_NO_P8) lower on
    the host through the same call; one result object serves batch after
    batch of different shapes."""
    wire = wire_of(2, 500, 3)
    dev, host = lower_both(dl, wire, p8=False)
    assert_same(dev, host)
    assert dl.host_count == 500
    lw = _lib.Lowered.empty()
    for cfg, n, seed in ((2, 3000, 1), (3, 5000, 2), (2, 700, 3), (6, 2000, 4)):
        w = wire_of(cfg, n, seed)
        dl.lower(_lib.Wire32Arrays(w), lw)
        assert_same(lw, _lib.Lowered(w, narrow=True, pinned=True, packed=True))


@pytest.mark.gpu
def test_device_lowered_batch_solves_like_host(dl):
    """The device-lowered batch goes to dp_submit as it lies (page-locked,
    staged forms) and solves to the host-lowered batch's results."""
    wire = wire_of(2, 4000, 9)
    dev, host = lower_both(dl, wire)
    ctx = dl.ctx
    a = ctx.submit(dev.rec_off, dev.rec).wait()
    b = ctx.submit(host.rec_off, host.rec).wait()
    for k in ("status", "flags", "installed", "core_len", "core"):
        np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.gpu
def test_device_lowering_malformed_wire(dl):
    """A malformed problem fails the whole call, as dp_lower_into does."""
    wire = wire_of(2, 50, 4)
    bad = _lib.WireArrays(**{k: v.copy() for k, v in wire.a.items() if k != "str_bytes"},
                          str_bytes=wire.a["str_bytes"][:-1].tobytes())
    bad.a["con_arg"][5] = len(bad.a["str_off"]) + 3  # a string index past the table
    with pytest.raises(ValueError, match="malformed"):
        _lib.Lowered(bad, narrow=True, packed=True)
    with pytest.raises(ValueError, match="malformed"):
        dl.lower(_lib.Wire32Arrays(bad))
    # the object still works after a failed call
    dev, host = lower_both(dl, wire)
    assert_same(dev, host)


def test_device_lowering_entry_points_refuse_null():
    """Without a context the entry points fail cleanly (no device touched):
    dp_dlower_new(NULL) gives NULL with a reason, dp_lower_device(NULL, ...)
    -1."""
    L = _lib.lib()
    assert not L.dp_dlower_new(None)
    assert b"no context" in L.dp_last_global_error()
    w32 = _lib.Wire32Arrays(wire_of(2, 3, 1))
    ws = w32.struct()
    lw = _lib.Lowered.empty()
    assert L.dp_lower_device(None, ctypes.byref(ws), lw._flags, lw._owner.h) == -1
    assert b"malformed" in L.dp_last_global_error()


@pytest.mark.gpu
def test_device_lowering_inconsistent_counts(dl):
    """The compact wire's counts must add up to each problem's ranges: a
    variable claiming one constraint more (or a constraint one argument more)
    makes the batch malformed, as dp_lower_into reports a malformed wire;
    the kernel leaves such a problem to the host, which reports it."""
    wire = wire_of(2, 200, 6)
    for key in ("var_ncon", "con_nargs"):
        w32 = _lib.Wire32Arrays(wire)
        w32.a[key][5] += 1
        with pytest.raises(ValueError, match="malformed"):
            dl.lower(w32)
    dev, host = lower_both(dl, wire)
    assert_same(dev, host)


@pytest.mark.gpu
def test_solve_wire_takes_the_compact_wire(dl):
    """sat.solve_wire (SolveBatch's wire-to-results half) lowers a compact
    wire on the GPU: the same records and results as from the 64-bit wire."""
    wire = wire_of(2, 3000, 12)
    lw_h, rh = sat.solve_wire(wire, dl.ctx)
    rec_h, off_h = lw_h.rec.copy(), lw_h.rec_off.copy()
    rh = {k: v.copy() for k, v in rh.items()}
    lw_d, rd = sat.solve_wire(_lib.Wire32Arrays(wire), dl.ctx)
    np.testing.assert_array_equal(lw_d.rec_off, off_h)
    np.testing.assert_array_equal(lw_d.rec, rec_h)
    for k in ("status", "flags", "installed", "core_len", "core", "steps"):
        np.testing.assert_array_equal(rd[k], rh[k])
