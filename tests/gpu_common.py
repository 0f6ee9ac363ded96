"""Shared helpers for the -m gpu tests (run on the MI355X box)."""
import numpy as np

from deppy_amd import _lib


def lowered_config(config, n, seed, narrow=False, pinned=False, packed=False, p8=True):
    """Synthetic catalogs (SURVEY §8(d) generator) lowered by dp_lower;
    narrow: records that fit 16 bits in the DP_FMT_U16 form (packed: the
    DP_FMT_P16D / DP_FMT_P16 forms where they apply); pinned: in page-locked memory (with a
    GPU)."""
    w = _lib.generate(config, n, seed)
    return _lib.Lowered(_lib.WireArrays(**{k: w[k] for k in (
        "prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off", "con_arg",
        "str_off")}, str_bytes=w["str_bytes"].tobytes()), narrow=narrow or packed, pinned=pinned,
        packed=packed, p8=p8)


def corrupt16(rec_off, rec, p, kind):
    """Make 16-bit record p malformed in place: 'lit' a clause literal past
    2*nv, 'off' decreasing clause offsets, 'run' an AtMost row whose variable
    positions are not one run (needs a row of >= 3 positions; returns False
    when there is none)."""
    r = rec[rec_off[p]:rec_off[p + 1]]
    assert r[13] == 1
    u = r[16:].view(np.uint16)
    nv, nc, nk, ncl = int(r[1]), int(r[2]), int(r[3]), int(r[7])
    if kind == "lit":
        u[nc + 1] = 2 * nv + 3
    elif kind == "off":
        u[1] = int(u[2]) + 1
    else:
        co = nc + 1 + ncl + nc
        cl = co + nk + 1
        for k in range(nk):
            a, b = int(u[co + k]), int(u[co + k + 1])
            if b - a >= 3 and u[cl + a] != u[cl + a + 1]:
                u[cl + a + 2] = u[cl + a]  # x y x: two runs of x
                return True
        return False
    return True


def implied_choices(nv, clause_off, clause_lits, src):
    """DP_FMT_P16D's choice lists (include/deppy_hip.h), restated: dependency
    rows (two or more literals, the first negative, the rest positive) in row
    order; src[k] == 0: list k = the variables after the first literal of the
    next one; src[k] = d: list k repeats list k - d; var_choice_off counts the
    lists per subject (the first literal's variable)."""
    dep = [r for r in range(len(clause_off) - 1)
           if clause_off[r + 1] - clause_off[r] >= 2 and clause_lits[clause_off[r]] & 1
           and not np.any(clause_lits[clause_off[r] + 1:clause_off[r + 1]] & 1)]
    per_var = np.zeros(nv, np.int64)
    co, chl, rows, j = [0], [], [], 0
    for s in src:
        row = dep[j] if s == 0 else rows[len(rows) - int(s)]
        j += s == 0
        rows.append(row)
        lits = clause_lits[clause_off[row]:clause_off[row + 1]]
        per_var[lits[0] >> 1] += 1
        chl.extend(int(x) >> 1 for x in lits[1:])
        co.append(len(chl))
    assert j == len(dep)
    vco = np.concatenate([[0], np.cumsum(per_var)])
    return vco.astype(np.int32), np.array(co, np.int32), np.array(chl, np.int32)


def unpack_p8(r):
    """The DP_FMT_P16D record a DP_FMT_P8D one encodes (include/deppy_hip.h),
    restated independently of the library: 8-bit variables with their sign
    and bit-8 planes, byte or nibble lengths, the nonzero list sources by a
    bit mask, then the identity mask."""
    nv, nc, nk, nch, na, nid, ncl, nkl = (int(r[i]) for i in range(1, 9))
    f = int(r[14]) & 0xff
    b = r[16:].view(np.uint8)
    at = 0

    def take(n):
        nonlocal at
        x = b[at:at + n]
        at += n
        return x

    def bits(n):
        return np.unpackbits(take((n + 7) // 8), bitorder="little")[:n].astype(np.int32)

    cv, kv, av = take(ncl).astype(np.int32), take(nkl).astype(np.int32), take(na).astype(np.int32)
    kb = np.ones(nk, np.int32) if f & 1 else take(nk).astype(np.int32)
    neg = bits(ncl)
    if f & 2:
        cv, kv, av = cv + 256 * bits(ncl), kv + 256 * bits(nkl), av + 256 * bits(na)
    if f & 4:
        nb = take((nc + nk + 1) // 2)
        lens = np.stack([nb & 15, nb >> 4], axis=1).reshape(-1)[:nc + nk]
    else:
        lens = take(nc + nk)
    nz = bits(nch).astype(bool)
    src = np.zeros(nch, np.uint8)
    src[nz] = take(int(nz.sum()))
    mask = take((nid + 7) // 8)
    u16 = np.concatenate([2 * cv + neg, kv, kb, av]).astype(np.uint16).tobytes()
    u16 += bytes((-len(u16)) % 16)
    body = u16 + np.asarray(lens, np.uint8).tobytes() + src.tobytes() + mask.tobytes()
    body += bytes((-len(body)) % 4)
    head = np.asarray(r[:16], np.int32).copy()
    head[13], head[14] = 5, 0
    return np.concatenate([head, np.frombuffer(body, np.int32)])


def unpack_p16(r):
    """The int32 form of one DP_FMT_P16 / DP_FMT_P16D (or DP_FMT_P8D, through
    unpack_p8) record (include/deppy_hip.h), restated here independently of
    the library's dp_rec_widen."""
    if int(r[13]) == 6:
        r = unpack_p8(r)
    nv, nc, nk, nch, na, nid, ncl, nkl, nchl, words = (int(r[i]) for i in range(1, 11))
    derived = int(r[13]) == 5
    u = r[16:].view(np.uint16)
    o, parts16 = 0, []
    for n in (ncl, nkl, nk, 0 if derived else nchl, na):
        parts16.append(u[o:o + n].astype(np.int32))
        o += n
    cl, kl, kb, chl, anc = parts16
    tail_at = (2 * o + 15) // 16 * 16
    t = r[16:].view(np.uint8)[tail_at:]
    offs, o = [], 0
    for n in ((nc, nk) if derived else (nc, nk, nv, nch)):
        offs.append(np.concatenate([[0], np.cumsum(t[o:o + n].astype(np.int32))]).astype(np.int32))
        o += n
    src = t[o:o + nch] if derived else None
    o += nch if derived else 0
    bits = np.unpackbits(t[o:o + (nid + 7) // 8], bitorder="little")[:nid].astype(bool)
    ids = np.arange(nid, dtype=np.int32)
    cid, kid = ids[~bits], ids[bits]
    if derived:
        vco, co, chl = implied_choices(nv, offs[0], cl, src)
        offs += [vco, co]
    out = np.concatenate([r[:16], offs[0], cl, cid, offs[1], kl, kb, kid, offs[2], offs[3], chl, anc]).astype(np.int32)
    out[13] = 0
    assert len(out) == words
    return out


def pack_p16(r32):
    """The DP_FMT_P16 form (explicit choice lists) of an int32 record that
    allows it, padded to 16 bytes -- how a producer that does not derive
    choice lists packs a record (the library's lowering emits DP_FMT_P16D when
    it can)."""
    nv, nc, nk, nch, na, nid, ncl, nkl, nchl, words = (int(r32[i]) for i in range(1, 11))
    o = 16
    clause_off = r32[o:o + nc + 1]; o += nc + 1
    clause_lits = r32[o:o + ncl]; o += ncl
    o += nc  # clause_id (ascending, the mask's clear bits)
    card_off = r32[o:o + nk + 1]; o += nk + 1
    card_lits = r32[o:o + nkl]; o += nkl
    card_bound = r32[o:o + nk]; o += nk
    card_id = r32[o:o + nk]; o += nk
    vco = r32[o:o + nv + 1]; o += nv + 1
    co = r32[o:o + nch + 1]; o += nch + 1
    chl = r32[o:o + nchl]; o += nchl
    anc = r32[o:o + na]
    u16 = np.concatenate([clause_lits, card_lits, card_bound, chl, anc]).astype(np.uint16).tobytes()
    u16 += bytes((-len(u16)) % 16)
    mask = np.zeros(nid, bool)
    mask[card_id] = True
    tail = np.concatenate([np.diff(x) for x in (clause_off, card_off, vco, co)]).astype(np.uint8).tobytes()
    tail += np.packbits(mask, bitorder="little").tobytes()
    body = u16 + tail
    body += bytes((-(64 + len(body))) % 16)
    head = np.asarray(r32[:16], np.int32).copy()
    head[13] = 3
    return np.concatenate([head, np.frombuffer(body, np.int32)])


def widen(rec_off, rec):
    """A batch with every 16-bit-form record widened to int32 (-> rec_off, rec)."""
    parts, offs = [], [0]
    for p in range(len(rec_off) - 1):
        r = rec[rec_off[p]:rec_off[p + 1]]
        if len(r) and r[13] in (3, 5, 6):
            r = unpack_p16(r)
        elif len(r) and r[13] == 1:
            words = int(r[10])
            body = r[16:].view(np.uint16)[:words - 16].astype(np.int32)
            r = np.concatenate([r[:16], body])
            r[13] = 0
        elif len(r):
            r = r[:int(r[10])].copy()  # (DP_LOWER_NARROW pads records to 16 bytes)
            r[13] = 0  # (DP_FMT_I32W: the watch lists dropped)
        parts.append(np.asarray(r, np.int32))
        offs.append(offs[-1] + len(r))
    return np.array(offs, np.int64), (np.concatenate(parts) if parts else np.zeros(0, np.int32))


def compare_results(g, o, n, rec_off=None, rec=None, only=None):
    """Bit-exact comparison of GPU and oracle dp_result dicts (status, flags,
    steps, installed bitmap, core); returns the mismatches.  only: the
    problems to compare (default: 0..n-1)."""
    bad = []
    for p in (range(n) if only is None else only):
        if g["status"][p] != o["status"][p] or g["flags"][p] != o["flags"][p] \
                or g["steps"][p] != o["steps"][p]:
            bad.append((p, "status/flags/steps", int(g["status"][p]), int(o["status"][p]),
                        int(g["flags"][p]), int(o["flags"][p]), int(g["steps"][p]), int(o["steps"][p])))
            continue
        a0, a1 = g["inst_off"][p], g["inst_off"][p + 1]
        if not np.array_equal(g["installed"][a0:a1], o["installed"][a0:a1]):
            bad.append((p, "installed"))
            continue
        c0 = g["core_off"][p]
        cl = int(g["core_len"][p])
        if cl != o["core_len"][p] or not np.array_equal(g["core"][c0:c0 + cl], o["core"][c0:c0 + cl]):
            bad.append((p, "core"))
    return bad


def wide_problems(seed, n, nvs):
    """Problems of nv variables each (nv drawn from nvs): Dependencies on
    far-apart candidates, Conflicts, Mandatory anchors, AtMost rows with
    bounds 1 and 2, and (in every other problem) a Dependency of 20
    candidates -- so their DP_FMT_P8D records use the bit-8 planes (257..512
    variables), byte bounds and byte lengths; past 512 variables they stay
    DP_FMT_P16D."""
    from deppy_amd import sat
    from tests.test_lowering import V
    rng = np.random.default_rng(seed)
    out = []
    for q in range(n):
        nv = int(nvs[q % len(nvs)])
        names = ["w%d" % i for i in range(nv)]
        vs = []
        for i in range(nv):
            cons = []
            u = rng.random()
            if u < 0.05:
                cons.append(sat.Mandatory())
            if rng.random() < 0.3:
                m = int(rng.integers(1, 5))
                cons.append(sat.Dependency(*[names[j] for j in rng.choice(nv, m, replace=False) if j != i]))
            if rng.random() < 0.1:
                j = int(rng.integers(0, nv))
                if j != i:
                    cons.append(sat.Conflict(names[j]))
            if i % 20 == 7:
                ids = [names[j] for j in rng.choice(nv, int(rng.integers(3, 7)), replace=False)]
                cons.append(sat.AtMost(int(rng.integers(1, 3)), *ids))
            if i == 3 and q % 2 == 0:
                cons.append(sat.Dependency(*[names[j] for j in rng.choice(nv, 20, replace=False) if j != i]))
            vs.append(V(names[i], *cons))
        out.append(vs)
    return out


def p8_sections(r):
    """Byte offsets of a DP_FMT_P8D record's sections (from the body's start;
    include/deppy_hip.h), and its count of nonzero list sources."""
    nv, nc, nk, nch, na, nid, ncl, nkl = (int(r[i]) for i in range(1, 9))
    f = int(r[14]) & 0xff
    S, at = {}, 0
    for name, n in (("cvar", ncl), ("kvar", nkl), ("avar", na), ("bound", 0 if f & 1 else nk),
                    ("neg", (ncl + 7) // 8), ("chi", (ncl + 7) // 8 if f & 2 else 0),
                    ("khi", (nkl + 7) // 8 if f & 2 else 0), ("ahi", (na + 7) // 8 if f & 2 else 0),
                    ("lens", (nc + nk + 1) // 2 if f & 4 else nc + nk), ("srcnz", (nch + 7) // 8)):
        S[name] = at
        at += n
    S["srcval"] = at
    b = np.asarray(r[16:], np.int32).view(np.uint8)
    S["nz"] = int(np.unpackbits(b[S["srcnz"]:S["srcnz"] + (nch + 7) // 8], bitorder="little")[:nch].sum())
    S["mask"] = at + S["nz"]
    return S
