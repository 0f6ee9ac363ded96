"""Host-side parts of the host-to-host pipeline (runtime.cpp), on the CPU.

dp_submit cuts a batch into chunks, stages every chunk's records (16-bit form
for the LDS path, with dp_rec_validate's checks fused in), and stitches each
chunk's results back into the caller's dp_result by problem index, with the
explanations read through a per-chunk pool.  These tests run the same code
through the library's host-only hooks, with no GPU: the staging round trip
must reproduce every record, the stitching of synthetic per-problem results
must put every value at its problem, for any chunking, and the per-device
partition must cover the batch contiguously.
"""
import numpy as np
import pytest

from deppy_amd import _lib
from tests.gpu_common import lowered_config


def _bounds_clamped(rec_off, rec):
    """The records with every AtMost bound over its row length set to the row
    length (how the 16-bit staging stores them; the same row)."""
    out = rec.copy()
    for p in range(len(rec_off) - 1):
        r = out[rec_off[p]:rec_off[p + 1]]
        nc, nk, ncl, nkl = int(r[2]), int(r[3]), int(r[7]), int(r[8])
        co = 16 + nc + 1 + ncl + nc
        cb = co + nk + 1 + nkl
        for k in range(nk):
            r[cb + k] = min(int(r[cb + k]), int(r[co + k + 1] - r[co + k]))
    return out


@pytest.mark.parametrize("config,n", [(2, 300), (3, 2000), (5, 120)])
@pytest.mark.parametrize("chunk", [1, 7, 4096])
def test_stage_roundtrip(config, n, chunk):
    lw = lowered_config(config, n, 77)
    out, firsts = _lib.stage_roundtrip(lw.rec_off, lw.rec, chunk_problems=chunk)
    assert np.array_equal(out, _bounds_clamped(lw.rec_off, lw.rec))
    assert firsts[0] == 0 and np.all(np.diff(firsts) > 0) and np.all(np.diff(firsts) <= chunk)
    assert len(firsts) == -(-n // chunk)


def test_stage_roundtrip_int32_path():
    # forced multi-wave placement stages int32 copies (dp_rec_validate path)
    lw = lowered_config(2, 50, 5)
    out, _ = _lib.stage_roundtrip(lw.rec_off, lw.rec, flags=_lib.OPT_FORCE_GROUP, chunk_problems=16)
    assert np.array_equal(out, lw.rec)


def test_stage_chunk_bytes_bound():
    lw = lowered_config(2, 200, 9)
    words = np.diff(lw.rec_off)
    cap = int(words.max()) * 4 * 10  # ten of the largest records
    _, firsts = _lib.stage_roundtrip(lw.rec_off, lw.rec, chunk_bytes=cap)
    bounds = list(firsts) + [len(words)]
    for a, b in zip(bounds[:-1], bounds[1:]):
        assert b - a == 1 or 4 * int(lw.rec_off[b] - lw.rec_off[a]) <= cap


def test_stage_rejects_malformed():
    lw = lowered_config(2, 20, 3)
    rec = lw.rec.copy()
    r0 = int(lw.rec_off[5])
    nc, ncl = int(rec[r0 + 2]), int(rec[r0 + 7])
    rec[r0 + 16 + nc + 1] = 2 * int(rec[r0 + 1]) + 3  # a clause literal past 2*nv
    with pytest.raises(ValueError):
        _lib.stage_roundtrip(lw.rec_off, rec)
    rec = lw.rec.copy()
    rec[r0 + 16 + 1] = rec[r0 + 16 + 2] + 1  # clause offsets not monotone
    if ncl:
        with pytest.raises(ValueError):
            _lib.stage_roundtrip(lw.rec_off, rec)


def _expected(lw):
    n = lw.n
    nv = lw.rec[lw.rec_off[:-1] + 1].astype(np.int64)
    nid = lw.rec[lw.rec_off[:-1] + 6].astype(np.int64)
    ref = _lib.result_arrays(lw.rec_off, lw.rec)
    for p in range(n):
        unsat = p % 3 == 0 and nid[p] > 0
        ref["status"][p] = -1 if unsat else 1
        ref["flags"][p] = p & 0xff
        ref["steps"][p] = 7 * p
        a, b = int(ref["inst_off"][p]), int(ref["inst_off"][p + 1])
        ref["installed"][a:b] = (np.uint32((p * 2654435761) & 0xffffffff) ^ np.arange(b - a, dtype=np.uint32))
        cl = min(int(nid[p]), 1 + p % 4) if unsat else 0
        ref["core_len"][p] = cl
        c0 = int(ref["core_off"][p])
        ref["core"][c0:c0 + cl] = [(p + j) % int(nid[p]) for j in range(cl)]
    return ref


@pytest.mark.parametrize("chunk", [1, 3, 64, 4096])
def test_stitching_any_chunking(chunk):
    lw = lowered_config(3, 500, 21)
    got = _lib.stitch_selftest(lw.rec_off, lw.rec, chunk)
    ref = _expected(lw)
    for k in ("status", "flags", "steps", "installed", "core_len"):
        assert np.array_equal(got[k][:lw.n], ref[k][:lw.n]), k
    for p in range(lw.n):
        c0, cl = int(ref["core_off"][p]), int(ref["core_len"][p])
        assert np.array_equal(got["core"][c0:c0 + cl], ref["core"][c0:c0 + cl]), p


@pytest.mark.parametrize("nd", [1, 2, 3, 8])
def test_partition_covers_batch(nd):
    lw = lowered_config(2, 101, 4)
    cut = _lib.partition(lw.rec_off, nd)
    assert cut[0] == 0 and cut[-1] == lw.n and np.all(np.diff(cut) >= 0)
    if nd <= lw.n:
        words = [int(lw.rec_off[cut[d + 1]] - lw.rec_off[cut[d]]) for d in range(nd)]
        assert max(words) <= int(lw.rec_off[-1]) / nd + int(np.diff(lw.rec_off).max())


@pytest.mark.parametrize("config,n", [(2, 200), (3, 1000), (5, 80), (4, 1)])
def test_narrow_lowering_is_the_16bit_form(config, n):
    """dp_lower_into(DP_LOWER_NARROW) emits exactly the int32 records, in the
    DP_FMT_U16 form wherever they fit 16 bits; every record validates."""
    from tests.gpu_common import widen
    a = lowered_config(config, n, 17)
    b = lowered_config(config, n, 17, narrow=True)
    off, rec = widen(b.rec_off, b.rec)
    np.testing.assert_array_equal(off, a.rec_off)
    np.testing.assert_array_equal(rec, a.rec)
    for p in range(n):
        r = b.record(p)
        # 16-bit for one-wavefront problems; multi-wave ones as plain int32
        # (the device builds their watch lists, layout.hpp DEV_WATCH_VARS)
        assert int(r[13]) in ((1, 0) if config == 5 else (1,) if config != 4 else (0,))
        assert _lib.lib().dp_rec_validate(np.ascontiguousarray(r).ctypes.data_as(_lib.c_i32p), len(r)) == 0
    np.testing.assert_array_equal(b.ident_var, a.ident_var)
    assert b.rec_off[-1] <= a.rec_off[-1]


@pytest.mark.parametrize("flags", [0, _lib.OPT_FORCE_GROUP])
def test_stage_roundtrip_narrow_source(flags):
    lw = lowered_config(2, 120, 23, narrow=True)
    out, _ = _lib.stage_roundtrip(lw.rec_off, lw.rec, flags=flags, chunk_problems=50)
    np.testing.assert_array_equal(out, lw.rec)


def test_oracle_reads_narrow_records():
    from oracle import oracle
    a = lowered_config(5, 60, 29)
    b = lowered_config(5, 60, 29, narrow=True)
    oa = oracle.solve_batch(a.rec_off, a.rec)
    ob = oracle.solve_batch(b.rec_off, b.rec)
    for k in ("status", "flags", "installed", "core", "core_len", "steps"):
        np.testing.assert_array_equal(oa[k], ob[k])


def test_validate_rejects_malformed_narrow():
    lw = lowered_config(2, 3, 31, narrow=True)
    r = np.ascontiguousarray(lw.record(1)).copy()
    u = r[16:].view(np.uint16)
    nc, ncl = int(r[2]), int(r[7])
    u[nc + 1] = 2 * int(r[1]) + 5  # first clause literal past 2*nv
    assert _lib.lib().dp_rec_validate(r.ctypes.data_as(_lib.c_i32p), len(r)) != 0


@pytest.mark.parametrize("config,n", [(2, 150), (4, 1), (5, 90)])
def test_narrow_records_on_16_byte_boundaries(config, n):
    """DP_LOWER_NARROW starts every record on a 16-byte boundary (the staged
    form as it is, so a page-locked batch needs no staging); the padding is
    zero and outside the record.  Without a GPU, DP_LOWER_PINNED falls back
    to ordinary memory."""
    b = lowered_config(config, n, 37, narrow=True, pinned=True)
    assert np.all(b.rec_off % 4 == 0)
    assert b.rec.ctypes.data % 16 == 0
    for p in range(n):
        r = b.record(p)
        nv, ncl, nkl = int(r[1]), int(r[7]), int(r[8])
        phys = (16 + (int(r[10]) - 15) // 2 if r[13] == 1 else int(r[10]) if r[13] == 0
                else int(r[10]) + 2 * nv + 1 + ncl + nkl)
        assert len(r) == (phys + 3) // 4 * 4 and not np.any(r[phys:])
    import torch
    if not torch.cuda.is_available():
        assert not b.pinned


# ---------------------------------------------------------------------------
# DP_FMT_P16: the packed 16-bit form (byte lengths + identity mask)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("config,n", [(2, 200), (3, 800), (5, 60), (4, 1)])
def test_packed_lowering_is_the_int32_record(config, n):
    """dp_lower_into(DP_LOWER_PACKED) emits exactly the int32 records (widened
    by an independent restatement of the format), in the DP_FMT_P16 form
    wherever it applies; dp_rec_widen and dp_rec_validate agree."""
    from tests.gpu_common import unpack_p16, widen
    a = lowered_config(config, n, 17)
    b = lowered_config(config, n, 17, packed=True)
    off, rec = widen(b.rec_off, b.rec)
    np.testing.assert_array_equal(off, a.rec_off)
    np.testing.assert_array_equal(rec, a.rec)
    fmt = b.rec[b.rec_off[:-1] + 13]
    if config in (2, 3):
        # the generated catalogs' dependency rows imply their choice lists;
        # DP_FMT_P8D up to 512 variables (all of them: config 2 peaks near 300)
        assert np.all(fmt == 6)
        c = lowered_config(config, n, 17, packed=True, p8=False)
        assert np.all(c.rec[c.rec_off[:-1] + 13] == 5)
        assert b.rec_off[-1] < 0.67 * c.rec_off[-1], (b.rec_off[-1], c.rec_off[-1])
    assert np.all(b.rec_off % 4 == 0)
    L = _lib.lib()
    for p in range(n):
        r = np.ascontiguousarray(b.record(p))
        out = np.zeros(int(r[10]), np.int32)
        assert L.dp_rec_widen(r.ctypes.data_as(_lib.c_i32p), len(r), out.ctypes.data_as(_lib.c_i32p)) == 0
        np.testing.assert_array_equal(out, a.record(p))
        assert L.dp_rec_validate(r.ctypes.data_as(_lib.c_i32p), len(r)) == 0
        if r[13] in (3, 5, 6):
            np.testing.assert_array_equal(unpack_p16(r), a.record(p))


def test_packed_malformed_is_rejected():
    """A mask with the wrong number of AtMost identities, lengths that do not
    sum to the row total, an out-of-range literal, dependency rows that no
    longer imply the header's choice lists (DP_FMT_P16D): dp_rec_validate
    rejects each (the kernel checks the same, tests/test_gpu_parity.py)."""
    b = lowered_config(2, 4, 41, packed=True, p8=False)
    L = _lib.lib()
    r0 = np.ascontiguousarray(b.record(1)).copy()
    assert r0[13] == 5
    nv, nc, nk, nch, na, nid, ncl, nkl, nchl = (int(r0[i]) for i in range(1, 10))
    nu16 = ncl + nkl + nk + na
    tail = (2 * nu16 + 15) // 16 * 16
    def bad(r):
        return L.dp_rec_validate(np.ascontiguousarray(r).ctypes.data_as(_lib.c_i32p), len(r)) != 0
    r = r0.copy(); t = r[16:].view(np.uint8); t[tail + nc + nk + nch] ^= 1            # mask: one bit flipped
    assert bad(r)
    r = r0.copy(); t = r[16:].view(np.uint8); t[tail] += 1                           # clause lengths: sum != ncl
    assert bad(r)
    r = r0.copy(); r[16:].view(np.uint16)[0] = 2 * nv + 1                             # clause literal past 2nv
    assert bad(r)
    r = r0.copy(); r[9] -= 1                                                          # nchl: one choice short
    assert bad(r)
    # a dependency row's first literal made positive: one list fewer than nch
    u = r0[16:].view(np.uint16)
    lens = r0[16:].view(np.uint8)[tail:tail + nc].astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)])
    dep = [a for a, e in zip(offs[:-1], offs[1:]) if e - a >= 2 and u[a] & 1 and not np.any(u[a + 1:e] & 1)]
    r = r0.copy(); r[16:].view(np.uint16)[dep[0]] ^= 1
    assert bad(r)
    assert not bad(r0)


def test_explicit_choice_packed_form():
    """DP_FMT_P16 (explicit choice lists, tests/gpu_common.pack_p16) widens to
    the int32 record through dp_rec_widen and the independent restatement,
    validates, and the oracle solves it like the int32 form."""
    from oracle import oracle
    from tests.gpu_common import pack_p16, unpack_p16
    a = lowered_config(2, 40, 23)
    L = _lib.lib()
    parts = []
    for p in range(a.n):
        r = pack_p16(a.record(p))
        assert r[13] == 3 and len(r) % 4 == 0
        out = np.zeros(int(r[10]), np.int32)
        assert L.dp_rec_widen(r.ctypes.data_as(_lib.c_i32p), len(r), out.ctypes.data_as(_lib.c_i32p)) == 0
        np.testing.assert_array_equal(out, a.record(p))
        np.testing.assert_array_equal(unpack_p16(r), a.record(p))
        assert L.dp_rec_validate(r.ctypes.data_as(_lib.c_i32p), len(r)) == 0
        parts.append(r)
    off = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.int64)
    ob = oracle.solve_batch(off, np.concatenate(parts))
    oa = oracle.solve_batch(a.rec_off, a.rec)
    for k in ("status", "flags", "installed", "core", "core_len", "steps"):
        np.testing.assert_array_equal(oa[k], ob[k])


def test_oracle_reads_packed_records():
    from oracle import oracle
    a = lowered_config(5, 60, 29)
    b = lowered_config(5, 60, 29, packed=True)
    oa = oracle.solve_batch(a.rec_off, a.rec)
    ob = oracle.solve_batch(b.rec_off, b.rec)
    for k in ("status", "flags", "installed", "core", "core_len", "steps"):
        np.testing.assert_array_equal(oa[k], ob[k])


def test_stage_roundtrip_packed_source():
    lw = lowered_config(2, 120, 23, packed=True)
    out, _ = _lib.stage_roundtrip(lw.rec_off, lw.rec, chunk_problems=50)
    np.testing.assert_array_equal(out, lw.rec)


def test_hw_queue_plan():
    """GPU_MAX_HW_QUEUES is read by HIP once, when it initialises: the binding
    raises it to 8 only while HIP is not up, and otherwise reports the queues
    HIP really runs with, so the runtime opens one lane stream per real queue
    (runtime.cpp lane_streams reads DEPPY_HW_QUEUES)."""
    plan = _lib.hw_queue_plan
    assert plan(None, False) == ("8", 8)
    assert plan("4", False) == ("8", 8)          # the boxes' exported default
    assert plan("16", False) == (None, 16)       # a larger setting stays
    assert plan("4", False, keep=True) == (None, 4)
    # HIP initialised before the binding: the setting cannot take effect any
    # more; the streams follow what HIP opened, not what the binding wants
    assert plan(None, True) == (None, 4)
    assert plan("4", True) == (None, 4)
    assert plan("8", True) == (None, 8)
    assert plan("junk", True) == (None, 4)
    import os
    q, at = os.environ["DEPPY_HW_QUEUES"].split("@")
    assert q == str(int(os.environ.get("GPU_MAX_HW_QUEUES", "4")))
    assert at == os.environ.get("GPU_MAX_HW_QUEUES", "")


def test_pipelined_solve_wire_stitching():
    """sat._solve_pipelined's result stitching (CPU): the per-sub-batch
    result dicts of a batch cut in three, stitched, equal the whole batch's
    (the oracle stands in for the device solve here), and the wire slices
    lower to the same records as the whole batch."""
    from deppy_amd import sat
    from oracle import oracle
    w = _lib.generate(5, 300, 77)
    wa = _lib.WireArrays(**{k: w[k] for k in ("prob_var_off", "var_id", "var_con_off", "con_kind", "con_n",
                                              "con_arg_off", "con_arg", "str_off")}, str_bytes=w["str_bytes"].tobytes())
    whole = _lib.Lowered(wa)
    full = oracle.solve_batch(whole.rec_off, whole.rec, 0, 4)
    cuts = [0, 97, 201, 300]
    subs, parts = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        lw = _lib.Lowered(wa.slice(a, b))
        np.testing.assert_array_equal(lw.rec, whole.rec[whole.rec_off[a]:whole.rec_off[b]])
        subs.append(oracle.solve_batch(lw.rec_off, lw.rec, 0, 4))
        parts.append((lw.n, lw.ident_off.copy(), lw.ident_var.copy(), lw.ident_con.copy(), lw.err.copy(), list(lw.msg)))
    got = sat._stitch_results(subs)
    for k in ("status", "flags", "core_len", "steps", "inst_off", "core_off"):
        np.testing.assert_array_equal(got[k], full[k][:len(got[k])], err_msg=k)
    n_inst, n_core = int(full["inst_off"][-1]), int(full["core_off"][-1])
    np.testing.assert_array_equal(got["installed"][:n_inst], full["installed"][:n_inst])
    for p in range(300):
        c0, c1 = int(full["core_off"][p]), int(full["core_off"][p]) + int(full["core_len"][p])
        np.testing.assert_array_equal(got["core"][c0:c1], full["core"][c0:c1])
    st = sat._Stitched(parts)
    np.testing.assert_array_equal(st.ident_off, whole.ident_off)
    np.testing.assert_array_equal(st.ident_var, whole.ident_var)
    np.testing.assert_array_equal(st.ident_con, whole.ident_con)
    np.testing.assert_array_equal(st.err, whole.err)
    assert n_core >= 0


# ---------------------------------------------------------------------------
# DP_FMT_P8D: DP_FMT_P16D in 8-bit variables + bit planes
# ---------------------------------------------------------------------------
def test_p8_wide_variables_and_flags():
    """Records of 257..512 variables take DP_FMT_P8D with the bit-8 planes,
    AtMost bounds of 2 their byte bounds, a 20-candidate Dependency byte
    lengths; past 512 variables the record stays DP_FMT_P16D.  Every record
    widens (dp_rec_widen and the restatement) to its int32 record."""
    from deppy_amd import sat
    from tests.gpu_common import unpack_p16, wide_problems
    probs = wide_problems(5, 8, [300, 512, 513, 200])
    wire = sat.encode_inputs(probs)
    a = _lib.Lowered(wire)
    b = _lib.Lowered(wire, narrow=True, packed=True)
    L = _lib.lib()
    flags = set()
    for p in range(a.n):
        r = np.ascontiguousarray(b.record(p))
        nv = int(r[1])
        assert int(r[13]) == (6 if nv <= 512 else 5), (p, nv, int(r[13]))
        if r[13] == 6:
            f = int(r[14]) & 0xff
            assert bool(f & 2) == (nv > 256)
            flags.add(f)
            assert (int(r[14]) >> 8) <= 4 * (len(r) - 16)
        out = np.zeros(int(r[10]), np.int32)
        assert L.dp_rec_widen(r.ctypes.data_as(_lib.c_i32p), len(r), out.ctypes.data_as(_lib.c_i32p)) == 0
        np.testing.assert_array_equal(out, a.record(p))
        np.testing.assert_array_equal(unpack_p16(r), a.record(p))
        assert L.dp_rec_validate(r.ctypes.data_as(_lib.c_i32p), len(r)) == 0
    assert any(f & 4 for f in flags) and any(not f & 4 for f in flags), flags  # nibble and byte lengths
    assert any(not f & 1 for f in flags), flags                                # byte bounds


def test_p8_is_the_p16d_record_in_fewer_bytes():
    """DP_FMT_P8D decodes (independent restatement) to exactly the
    DP_FMT_P16D record DP_LOWER_NO_P8 emits, and config 2's batch shrinks by
    at least a third."""
    from tests.gpu_common import unpack_p8
    a = lowered_config(2, 300, 19, packed=True, p8=False)
    b = lowered_config(2, 300, 19, packed=True)
    for p in range(a.n):
        r16, r8 = a.record(p), b.record(p)
        assert r16[13] == 5 and r8[13] == 6
        d = unpack_p8(np.ascontiguousarray(r8))
        np.testing.assert_array_equal(d, r16[:len(d)])
        assert not np.any(r16[len(d):])  # (the rest is padding)
    assert b.rec_off[-1] < 0.67 * a.rec_off[-1], (b.rec_off[-1], a.rec_off[-1])


def test_p8_malformed_is_rejected():
    """An unknown flag bit, a body byte count shorter than its sections, a
    list source marked nonzero that is zero, a variable past nv (the bit-8
    plane), lengths that do not sum to the row total: dp_rec_validate rejects
    each (the kernel checks the same, tests/test_gpu_parity.py)."""
    from tests.gpu_common import p8_sections
    b = lowered_config(2, 40, 43, packed=True)
    L = _lib.lib()

    def bad(r):
        return L.dp_rec_validate(np.ascontiguousarray(r).ctypes.data_as(_lib.c_i32p), len(r)) != 0
    p = next(p for p in range(b.n) if int(b.record(p)[14]) & 4 and int(b.record(p)[1]) < 256
             and p8_sections(b.record(p))["nz"] > 0)
    r0 = np.ascontiguousarray(b.record(p)).copy()
    assert r0[13] == 6 and not bad(r0)
    S = p8_sections(r0)
    r = r0.copy(); r[14] |= 64                                                        # unknown flag
    assert bad(r)
    r = r0.copy(); r[14] = (r[14] & 0xff) | ((S["srcval"] - 1) << 8)                 # body too short
    assert bad(r)
    r = r0.copy(); t = r[16:].view(np.uint8); t[S["srcval"]] = 0                     # a nonzero source is 0
    assert bad(r)
    r = r0.copy(); t = r[16:].view(np.uint8); t[0] = 255                             # variable past nv
    assert bad(r)
    r = r0.copy(); t = r[16:].view(np.uint8); t[S["lens"]] ^= 1                      # a row length off by one
    assert bad(r)
