"""Placement and code-object guard rails, on CPU.

- Each workload plans to the placement DESIGN.md §5 gives it
  (dp_plan_placements, the pipeline's own plan_chunk).  Round 5 added an
  identity bitset without budgeting it in the round table's LDS, and every
  OLM-scale catalog silently left M_SPLIT for M_HBM; these tests would have
  caught it.
- No shipped solve kernel spills VGPRs to scratch: the gfx950 code objects
  inside libdeppy_hip.so carry the compiler's counts in their AMDGPU metadata
  note.
"""
import os
import shutil
import struct
import subprocess
import tempfile

import numpy as np
import pytest

from deppy_amd import _lib
from tests.gpu_common import lowered_config

SPLIT, HBM, SPLIT4, LDS = _lib.PLACES.index("split"), _lib.PLACES.index("hbm"), \
    _lib.PLACES.index("split4"), _lib.PLACES.index("lds")


@pytest.mark.parametrize("seed", [31, 32])
def test_olm_scale_plans_split(seed):
    """Config 4 (OLM-scale, ~55k variables): one 8-wave workgroup with its
    per-variable and round state in LDS (M_SPLIT), never M_HBM."""
    lw = lowered_config(4, 3, seed, narrow=True, packed=True)
    assert min(int(lw.record(p)[1]) for p in range(lw.n)) > 50000
    place = _lib.plan_placements(lw.rec_off, lw.rec)
    assert (place == SPLIT).all(), place


def test_config2_plans_one_wavefront():
    lw = lowered_config(2, 500, 3, narrow=True, packed=True)
    place = _lib.plan_placements(lw.rec_off, lw.rec)
    assert (place == LDS).all(), np.bincount(place + 2)


def test_config5_placements():
    """Config 5 mixes sizes: the small catalogs run one wavefront each, the
    large ones multi-wave groups that keep their state in LDS; a 2000-catalog
    chunk holds too many mid-size catalogs for M_LDSG (placement.hpp)."""
    lw = lowered_config(5, 2000, 5, narrow=True, packed=True)
    place = _lib.plan_placements(lw.rec_off, lw.rec)
    assert set(np.unique(place).tolist()) <= {LDS, SPLIT4, SPLIT}, np.unique(place)
    assert (place == LDS).any() and (place == SPLIT4).any()


def test_forced_hbm_plans_hbm():
    lw = lowered_config(2, 50, 3)
    assert (_lib.plan_placements(lw.rec_off, lw.rec, _lib.OPT_FORCE_HBM) == HBM).all()


# ---------------------------------------------------------------------------
# gfx950 code objects: register spills
# ---------------------------------------------------------------------------
LLVM = "/opt/rocm/lib/llvm/bin"


def _bundles(path):
    """The amdgcn code objects of the clang offload bundles in the library's
    .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fb, path,
                        os.path.join(d, "x.so")], check=True)
        data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out, i = [], data.find(magic)
    while i >= 0:
        (n,) = struct.unpack_from("<Q", data, i + 24)
        o = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, o)
            o += 24
            triple = data[o:o + tl].decode()
            o += tl
            if "amdgcn" in triple and size:
                out.append((triple, data[i + off:i + off + size]))
        i = data.find(magic, i + 1)
    return out


def _kernels(elf):
    """amdhsa.kernels of a code object's NT_AMDGPU_METADATA note (msgpack)."""
    import msgpack
    (shoff,) = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    res = []
    for k in range(shnum):
        b = shoff + k * shentsize
        if struct.unpack_from("<I", elf, b + 4)[0] != 7:  # SHT_NOTE
            continue
        off, size = struct.unpack_from("<QQ", elf, b + 0x18)
        p = off
        while p < off + size:
            nsz, dsz, typ = struct.unpack_from("<III", elf, p)
            p += 12
            name = elf[p:p + nsz]
            p += (nsz + 3) & ~3
            desc = elf[p:p + dsz]
            p += (dsz + 3) & ~3
            if name.startswith(b"AMDGPU") and typ == 32:
                res += msgpack.unpackb(desc, raw=False, strict_map_key=False)["amdhsa.kernels"]
    return res


def code_object_kernels(path=_lib.LIB_PATH):
    ks = []
    for triple, elf in _bundles(path):
        assert triple.endswith("gfx950"), triple
        ks += _kernels(elf)
    return ks


@pytest.mark.skipif(shutil.which(os.path.join(LLVM, "llvm-objcopy")) is None, reason="no llvm-objcopy")
def test_no_vgpr_spills():
    """Every kernel of the product library keeps its live state in registers:
    no VGPR spill and no scratch (private segment).  A spill writes scratch
    per lane through the memory system: round 5's capped one-wavefront build
    spilled 13 VGPRs and config 3's fabric writes rose 8.7x."""
    ks = code_object_kernels()
    solve = [k for k in ks if "solve_kernel" in k[".name"]]
    assert len(solve) >= 6, [k[".name"] for k in ks]
    bad = [(k[".name"], k[".vgpr_count"], k[".vgpr_spill_count"], k[".private_segment_fixed_size"])
           for k in ks if k[".vgpr_spill_count"] or k[".private_segment_fixed_size"]]
    assert bad == [], bad


# ---------------------------------------------------------------------------
# dispatch order (runtime.cpp plan_chunk)
# ---------------------------------------------------------------------------
def _expected_lds_order(rec_off, rec, members, first_rel=0):
    """A one-wavefront launch's workgroup order, restated: cost classes
    (anchors, at most 15) costliest first, members in problem order within a
    class, each class dealt XCD-contiguously (workgroup b on XCD b % 8 takes
    the next of XCD (b % 8)'s contiguous range of the class)."""
    cls = {p: min(int(rec[rec_off[p] + 5]), 15) for p in members}
    srt = sorted(members, key=lambda p: (-cls[p], p))
    out = [None] * len(srt)
    pos = 0
    while pos < len(srt):
        end = pos
        while end < len(srt) and cls[srt[end]] == cls[srt[pos]]:
            end += 1
        slots = {x: [b for b in range(pos, end) if (b + first_rel) % 8 == x] for x in range(8)}
        at = pos
        for x in range(8):
            for k, b in enumerate(slots[x]):
                out[b] = srt[at + k]
            at += len(slots[x])
        pos = end
    return out


def test_plan_order_one_wavefront():
    """Config 2 (one launch of one-wavefront problems): the planned order is
    the costliest anchor class first, XCD-contiguous within each class."""
    lw = lowered_config(2, 3000, 7, narrow=True, packed=True)
    order, first = _lib.plan_order(lw.rec_off, lw.rec)
    assert list(first) == [0]
    assert list(order) == _expected_lds_order(lw.rec_off, lw.rec, list(range(lw.n)))


def test_plan_order_mixed_launches():
    """Config 5 (multi-wave launches first, then the one-wavefront ones):
    every problem once, each launch's members of one placement, and each
    one-wavefront launch in the restated order (its XCDs counted from its
    first workgroup)."""
    lw = lowered_config(5, 2000, 9, narrow=True, packed=True)
    place = _lib.plan_placements(lw.rec_off, lw.rec)
    order, first = _lib.plan_order(lw.rec_off, lw.rec)
    assert sorted(order.tolist()) == list(range(lw.n))
    bounds = list(first) + [lw.n]
    assert len(first) >= 2
    for a, b in zip(bounds[:-1], bounds[1:]):
        seg = order[a:b].tolist()
        kinds = set(place[seg].tolist())
        assert len(kinds) == 1, kinds
        if kinds == {LDS}:
            assert seg == _expected_lds_order(lw.rec_off, lw.rec, sorted(seg), first_rel=0), (a, b)


@pytest.mark.gpu
def test_ldsg_rule_counts_the_device_load():
    """M_LDSG holds a whole CU's LDS per catalog, so the pipeline puts
    mid-size catalogs there only while the device's M_LDSG problems in flight
    (every lane's chunk, not the new chunk's alone) stay within
    kLdsgMaxProblems (runtime.cpp start_chunk).  A batch of
    120 such catalogs alone goes to M_LDSG; 16 of them submitted at once
    mostly do not, and every result equals the one-job result."""
    ldsg = _lib.PLACES.index("ldsg")
    lw = lowered_config(5, 1500, 21)
    pl = _lib.plan_placements(lw.rec_off, lw.rec)
    pf = _lib.plan_placements(lw.rec_off, lw.rec, _lib.OPT_FORCE_LDSG)
    mid = [p for p in range(lw.n) if pl[p] != LDS and pf[p] == ldsg][:120]
    assert len(mid) == 120
    recs = [lw.rec[lw.rec_off[p]:lw.rec_off[p + 1]] for p in mid]
    rec = np.concatenate(recs).astype(np.int32)
    rec_off = np.concatenate([[0], np.cumsum([len(r) for r in recs])]).astype(np.int64)
    assert (_lib.plan_placements(rec_off, rec) == ldsg).all()
    ctx = _lib.Context(0, 1)
    try:
        ctx.stats(reset=True)
        one = ctx.submit(rec_off, rec).wait()
        assert ctx.stats(reset=True)["placed"]["ldsg"] == 120
        jobs = [ctx.submit(rec_off, rec) for _ in range(16)]
        outs = [j.wait() for j in jobs]
        st = ctx.stats(reset=True)["placed"]
        assert st["ldsg"] + st["split4"] == 16 * 120, st
        assert st["ldsg"] <= 8 * 120, st
        for o in outs:
            for k in ("status", "flags", "installed", "core_len", "core", "steps"):
                np.testing.assert_array_equal(o[k], one[k])
    finally:
        ctx.close()
