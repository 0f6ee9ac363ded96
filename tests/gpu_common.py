"""Shared helpers for the -m gpu tests (run on the MI355X box)."""
import numpy as np

from deppy_amd import _lib


def lowered_config(config, n, seed, narrow=False, pinned=False, packed=False):
    """Synthetic catalogs (SURVEY §8(d) generator) lowered by dp_lower;
    narrow: records that fit 16 bits in the DP_FMT_U16 form (packed: the
    DP_FMT_P16 form where it applies); pinned: in page-locked memory (with a
    GPU)."""
    w = _lib.generate(config, n, seed)
    return _lib.Lowered(_lib.WireArrays(**{k: w[k] for k in (
        "prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off", "con_arg",
        "str_off")}, str_bytes=w["str_bytes"].tobytes()), narrow=narrow or packed, pinned=pinned,
        packed=packed)


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


def unpack_p16(r):
    """The int32 form of one DP_FMT_P16 record (include/deppy_hip.h), restated
    here independently of the library's dp_rec_widen."""
    nv, nc, nk, nch, na, nid, ncl, nkl, nchl, words = (int(r[i]) for i in range(1, 11))
    u = r[16:].view(np.uint16)
    o, parts16 = 0, []
    for n in (ncl, nkl, nk, nchl, na):
        parts16.append(u[o:o + n].astype(np.int32))
        o += n
    cl, kl, kb, chl, anc = parts16
    tail_at = (2 * o + 15) // 16 * 16
    t = r[16:].view(np.uint8)[tail_at:]
    offs, o = [], 0
    for n in (nc, nk, nv, nch):
        offs.append(np.concatenate([[0], np.cumsum(t[o:o + n].astype(np.int32))]).astype(np.int32))
        o += n
    bits = np.unpackbits(t[o:o + (nid + 7) // 8], bitorder="little")[:nid].astype(bool)
    ids = np.arange(nid, dtype=np.int32)
    cid, kid = ids[~bits], ids[bits]
    out = np.concatenate([r[:16], offs[0], cl, cid, offs[1], kl, kb, kid, offs[2], offs[3], chl, anc]).astype(np.int32)
    out[13] = 0
    assert len(out) == words
    return out


def widen(rec_off, rec):
    """A batch with every 16-bit-form record widened to int32 (-> rec_off, rec)."""
    parts, offs = [], [0]
    for p in range(len(rec_off) - 1):
        r = rec[rec_off[p]:rec_off[p + 1]]
        if len(r) and r[13] == 3:
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


def compare_results(g, o, n, rec_off=None, rec=None):
    """Bit-exact comparison of GPU and oracle dp_result dicts; returns mismatches."""
    bad = []
    for p in range(n):
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
