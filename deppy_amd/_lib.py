"""ctypes binding of libdeppy_hip.so (include/deppy_hip.h).

This is the same C-ABI a Go caller binds through cgo.  The
library is built in-tree by deppy_amd/build.py; importing this module never
falls back to anything else: a missing library or a missing MI355X is an error.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libdeppy_hip.so")
# The pipeline runs one lane stream per hardware queue the HIP runtime opens,
# at most 8.  HIP opens GPU_MAX_HW_QUEUES queues (default 4; the GPU boxes
# export 4) once, when it initialises: measured on one box, config 2 host to
# host 20.9M res/s on 4 queues, 22.0M on 8 (kernel only 25.5M -> 27.0M), and
# 8 streams on 4 queues 20.9-21.2M.  So before HIP starts, the
# binding raises the setting to 8 (DEPPY_KEEP_HW_QUEUES=1 keeps the operator's
# value); once HIP is up (another library initialised it first) the setting
# can no longer take effect, and the runtime sizes its streams from the queues
# HIP actually runs with.  Either way DEPPY_HW_QUEUES tells dp_create that
# number (runtime.cpp lane_streams).
def _hsa_up() -> bool:
    """Has this process opened the ROCm kernel driver (HIP initialised)?"""
    try:
        fds = os.listdir("/proc/self/fd")
    except OSError:
        return False
    for fd in fds:
        try:
            if os.readlink("/proc/self/fd/" + fd) == "/dev/kfd":
                return True
        except OSError:
            pass
    return False


def hw_queue_plan(env_value, hsa_up: bool, keep: bool = False):
    """-> (value to set GPU_MAX_HW_QUEUES to, or None; queues HIP runs with).
    HIP reads the setting once, when it initialises (default 4)."""
    try:
        q = int(env_value) if env_value not in (None, "") else 4
    except ValueError:
        q = 4
    if hsa_up or keep or q >= 8:
        return None, q
    return "8", 8


def _plan_hw_queues() -> None:
    up = _hsa_up()
    env = os.environ.get("GPU_MAX_HW_QUEUES")
    set_to, q = hw_queue_plan(env, up, os.environ.get("DEPPY_KEEP_HW_QUEUES") == "1")
    if set_to is not None:
        os.environ["GPU_MAX_HW_QUEUES"] = set_to
    elif up and q < 8:
        import warnings
        warnings.warn("deppy_amd: HIP was initialised before the binding was imported, with %d hardware "
                      "queues; the pipeline runs %d lane streams per device (import deppy_amd first for 8)"
                      % (q, q), RuntimeWarning, stacklevel=3)
    # "q@s": HIP runs q queues, known while GPU_MAX_HW_QUEUES reads s (a child
    # process started with another setting sizes its streams from its own)
    os.environ["DEPPY_HW_QUEUES"] = "%d@%s" % (q, os.environ.get("GPU_MAX_HW_QUEUES", ""))


_plan_hw_queues()
# dp_opt_flag (include/deppy_hip.h): placement overrides
OPT_FORCE_GROUP = 1 << 0
OPT_FORCE_HBM = 1 << 1
OPT_FORCE_MID = 1 << 2
OPT_TINY_TABLE = 1 << 3
OPT_FORCE_LDSG = 1 << 4
OPT_SHARE_ORDINAL = 1 << 5  # test: every logical device of the context on first_device's GPU
# dp_flag bits used on the host
F_TRACE_TRUNCATED = 1 << 8
if os.environ.get("DEPPY_STAMPS") == "1":  # diagnostic phase-stamp build (scripts/ only)
    LIB_PATH = os.path.join(HERE, os.environ.get("DEPPY_STAMPS_LIB", "libdeppy_hip_stamps.so"))
elif os.environ.get("DEPPY_VARIANT_LIB"):  # a tagged release variant (measurement scripts only)
    LIB_PATH = os.path.join(HERE, os.environ["DEPPY_VARIANT_LIB"])

c_i32p = ctypes.POINTER(ctypes.c_int32)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_i8p = ctypes.POINTER(ctypes.c_int8)

# every entry point declared in include/deppy_hip.h
EXPORTS = [
    "dp_rec_validate", "dp_lower", "dp_lowered_free", "dp_lowered_num_problems",
    "dp_lowered_rec_off", "dp_lowered_rec", "dp_lowered_ident_off", "dp_lowered_ident_var",
    "dp_lowered_ident_con", "dp_lowered_error", "dp_result_layout", "dp_create", "dp_destroy",
    "dp_last_error", "dp_last_global_error", "dp_num_devices", "dp_lanes", "dp_solve", "dp_upload", "dp_run",
    "dp_launch", "dp_wait", "dp_download", "dp_resident_free", "dp_last_kernel_ms", "dp_gen_catalogs", "dp_gen_wire",
    "dp_gen_free", "dp_upload_traced", "dp_download_trace", "dp_solve_traced", "dp_lowered_errors",
    "dp_device_bytes", "dp_lower_into", "dp_lowered_new", "dp_lowered_exact_count", "dp_lowered_pinned", "dp_rec_widen", "dp_submit", "dp_job_wait", "dp_get_stats", "dp_stage_roundtrip",
    "dp_stitch_selftest", "dp_partition", "dp_build_info", "dp_get_device_stats", "dp_plan_placements",
    "dp_plan_order", "dp_dlower_new", "dp_dlower_free", "dp_lower_device", "dp_dlower_host_count",
    "dp_host_alloc", "dp_host_free",
]


class Wire(ctypes.Structure):
    _fields_ = [
        ("n_problems", ctypes.c_int32),
        ("prob_var_off", c_i64p),
        ("var_id", c_i64p),
        ("var_con_off", c_i64p),
        ("con_kind", c_i32p),
        ("con_n", c_i32p),
        ("con_arg_off", c_i64p),
        ("con_arg", c_i64p),
        ("n_strs", ctypes.c_int64),
        ("str_off", c_i64p),
        ("str_bytes", ctypes.c_char_p),
        ("interned", ctypes.c_int32),
    ]


class Wire32(ctypes.Structure):
    _fields_ = [
        ("n_problems", ctypes.c_int32),
        ("prob_var_off", c_i32p),
        ("prob_con_off", c_i32p),
        ("prob_arg_off", c_i32p),
        ("var_id", c_i32p),
        ("var_ncon", ctypes.POINTER(ctypes.c_uint16)),
        ("con_kn", c_i32p),
        ("con_nargs", ctypes.POINTER(ctypes.c_uint16)),
        ("con_arg", c_i32p),
        ("var_id16", ctypes.POINTER(ctypes.c_uint16)),
        ("con_arg16", ctypes.POINTER(ctypes.c_uint16)),
        ("n_strs", ctypes.c_int64),
        ("str_off", c_i64p),
        ("str_bytes", ctypes.c_char_p),
    ]


class Opts(ctypes.Structure):
    _fields_ = [("first_device", ctypes.c_int32), ("n_devices", ctypes.c_int32),
                ("step_budget", ctypes.c_int64), ("flags", ctypes.c_int32)]


class Stats(ctypes.Structure):
    _fields_ = [("problems", ctypes.c_int64), ("chunks", ctypes.c_int64), ("launches", ctypes.c_int64),
                ("kernel_ms", ctypes.c_double), ("h2d_bytes", ctypes.c_int64), ("d2h_bytes", ctypes.c_int64),
                ("rec_bytes", ctypes.c_int64), ("stage_ms", ctypes.c_double), ("plan_ms", ctypes.c_double), ("wait_ms", ctypes.c_double),
                ("scatter_ms", ctypes.c_double), ("direct_chunks", ctypes.c_int64),
                ("bcp_bytes", ctypes.c_int64), ("allocs", ctypes.c_int64),
                ("placed", ctypes.c_int64 * 5), ("placed_launches", ctypes.c_int64 * 5)]

# enum dp_place (include/deppy_hip.h), the index of Stats.placed
PLACES = ["lds", "split", "hbm", "split4", "ldsg"]


def _stats_dict(st) -> dict:
    d = {}
    for k, _ in Stats._fields_:
        v = getattr(st, k)
        d[k] = {PLACES[m]: int(v[m]) for m in range(5)} if k.startswith("placed") else v
    return d


class Batch(ctypes.Structure):
    _fields_ = [("n_problems", ctypes.c_int32), ("rec_off", c_i64p), ("rec", c_i32p)]


class Result(ctypes.Structure):
    _fields_ = [("status", c_i8p), ("flags", c_i32p), ("installed", c_u32p),
                ("inst_off", c_i64p), ("core", c_i32p), ("core_off", c_i64p),
                ("core_len", c_i32p), ("steps", c_i64p)]


_lib = None


def build_info(L=None) -> str:
    """The library's dp_build_info string ("sources=<digest> arch=gfx950"),
    or "" for a library without it (an older measurement variant)."""
    L = L or lib()
    if not hasattr(L, "dp_build_info"):
        return ""
    L.dp_build_info.restype = ctypes.c_char_p
    return L.dp_build_info().decode()


def _check_provenance(L) -> None:
    """The product library must be the one the tree's sources make: its
    embedded digest (build.py sources_digest) against the digest of the
    sources it runs beside.  Measurement variants (DEPPY_VARIANT_LIB, the
    stamps build) are other revisions or flags by design and are not
    checked."""
    if LIB_PATH != os.path.join(HERE, "libdeppy_hip.so"):
        return
    from deppy_amd import build as _build  # (sources only; nothing is compiled here)
    try:
        want = _build.sources_digest()
    except OSError as e:
        raise RuntimeError("deppy_amd: cannot check that %s was built from this tree: its sources are not "
                           "readable (%s); deploy deppy_amd/csrc and include/ beside the library" % (LIB_PATH, e)) from e
    got = build_info(L)
    if ("sources=%s " % want) not in got + " ":
        raise RuntimeError("deppy_amd: %s was built from other sources (%s; this tree: sources=%s); run "
                           "__graft_entry__.build() (python -m deppy_amd.build)" % (LIB_PATH, got or "no build info", want))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("deppy_amd: %s is missing; run __graft_entry__.build() "
                           "(python deppy_amd/build.py)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    _check_provenance(L)
    vp = ctypes.c_void_p
    L.dp_rec_validate.argtypes = [c_i32p, ctypes.c_int64]
    L.dp_rec_widen.argtypes = [c_i32p, ctypes.c_int64, c_i32p]
    L.dp_lower.argtypes = [ctypes.POINTER(Wire), ctypes.POINTER(vp)]
    L.dp_lowered_free.argtypes = [vp]
    L.dp_lower_into.argtypes = [ctypes.POINTER(Wire), ctypes.c_int32, vp]
    L.dp_lowered_new.restype = vp
    L.dp_lowered_exact_count.argtypes = [vp]
    L.dp_lowered_exact_count.restype = ctypes.c_int64
    L.dp_lowered_pinned.argtypes = [vp]
    L.dp_lowered_pinned.restype = ctypes.c_int32
    L.dp_lowered_num_problems.argtypes = [vp]
    for f in ("dp_lowered_rec_off", "dp_lowered_ident_off"):
        getattr(L, f).argtypes = [vp]
        getattr(L, f).restype = c_i64p
    for f in ("dp_lowered_rec", "dp_lowered_ident_var", "dp_lowered_ident_con"):
        getattr(L, f).argtypes = [vp]
        getattr(L, f).restype = c_i32p
    L.dp_lowered_error.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_char_p)]
    L.dp_lowered_errors.argtypes = [vp, c_i32p]
    L.dp_result_layout.argtypes = [ctypes.POINTER(Batch), c_i64p, c_i64p]
    L.dp_create.argtypes = [ctypes.POINTER(Opts)]
    L.dp_create.restype = vp
    L.dp_destroy.argtypes = [vp]
    L.dp_last_error.argtypes = [vp]
    L.dp_last_error.restype = ctypes.c_char_p
    L.dp_last_global_error.restype = ctypes.c_char_p
    L.dp_num_devices.argtypes = [vp]
    if hasattr(L, "dp_lanes"):  # (an older build loaded as a measurement variant may lack it)
        L.dp_lanes.argtypes = [vp]
        L.dp_lanes.restype = ctypes.c_int32
    L.dp_solve.argtypes = [vp, ctypes.POINTER(Batch), ctypes.POINTER(Result)]
    L.dp_upload.argtypes = [vp, ctypes.POINTER(Batch), ctypes.POINTER(vp)]
    L.dp_upload_traced.argtypes = [vp, ctypes.POINTER(Batch), ctypes.c_int32, ctypes.POINTER(vp)]
    L.dp_download_trace.argtypes = [vp, vp, c_i32p, c_i32p]
    L.dp_solve_traced.argtypes = [vp, ctypes.POINTER(Batch), ctypes.c_int32, ctypes.POINTER(Result),
                                  c_i32p, c_i32p]
    L.dp_submit.argtypes = [vp, ctypes.POINTER(Batch), ctypes.POINTER(Result), ctypes.POINTER(vp)]
    L.dp_job_wait.argtypes = [vp, vp]
    L.dp_get_stats.argtypes = [vp, ctypes.POINTER(Stats), ctypes.c_int32]
    L.dp_get_device_stats.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(Stats), ctypes.c_int32]
    L.dp_num_devices.restype = ctypes.c_int32
    L.dp_stage_roundtrip.argtypes = [ctypes.POINTER(Batch), ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                     c_i32p, c_i32p, ctypes.c_int32]
    L.dp_stitch_selftest.argtypes = [ctypes.POINTER(Batch), ctypes.c_int32, ctypes.POINTER(Result)]
    L.dp_partition.argtypes = [c_i64p, ctypes.c_int32, ctypes.c_int32, c_i32p]
    L.dp_run.argtypes = [vp, vp]
    L.dp_launch.argtypes = [vp, vp]
    L.dp_wait.argtypes = [vp, vp]
    L.dp_download.argtypes = [vp, vp, ctypes.POINTER(Result)]
    L.dp_resident_free.argtypes = [vp, vp]
    L.dp_last_kernel_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
    L.dp_gen_catalogs.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64]
    L.dp_gen_catalogs.restype = vp
    L.dp_gen_wire.argtypes = [vp]
    L.dp_gen_wire.restype = ctypes.POINTER(Wire)
    L.dp_gen_free.argtypes = [vp]
    L.dp_device_bytes.argtypes = [ctypes.POINTER(Batch), ctypes.c_int32, c_i64p, c_i64p]
    L.dp_dlower_new.argtypes = [vp]
    L.dp_dlower_new.restype = vp
    L.dp_dlower_free.argtypes = [vp]
    L.dp_lower_device.argtypes = [vp, ctypes.POINTER(Wire32), ctypes.c_int32, vp]
    L.dp_dlower_host_count.argtypes = [vp]
    L.dp_dlower_host_count.restype = ctypes.c_int64
    L.dp_host_alloc.argtypes = [ctypes.c_int64]
    L.dp_host_alloc.restype = vp
    L.dp_host_free.argtypes = [vp]
    L.dp_plan_placements.argtypes = [ctypes.POINTER(Batch), ctypes.c_int32, c_i8p]
    L.dp_plan_order.argtypes = [ctypes.POINTER(Batch), ctypes.c_int32, c_i32p, c_i32p]
    _lib = L
    return L


def _p(a, t):
    return a.ctypes.data_as(t)


# ---------------------------------------------------------------------------
# wire batches
# ---------------------------------------------------------------------------
class WireArrays:
    """numpy-backed dp_wire (keeps the arrays alive while C reads them)."""

    def __init__(self, prob_var_off, var_id, var_con_off, con_kind, con_n, con_arg_off, con_arg,
                 str_off, str_bytes, interned=True):
        self.a = dict(prob_var_off=np.ascontiguousarray(prob_var_off, np.int64),
                      var_id=np.ascontiguousarray(var_id, np.int64),
                      var_con_off=np.ascontiguousarray(var_con_off, np.int64),
                      con_kind=np.ascontiguousarray(con_kind, np.int32),
                      con_n=np.ascontiguousarray(con_n, np.int32),
                      con_arg_off=np.ascontiguousarray(con_arg_off, np.int64),
                      con_arg=np.ascontiguousarray(con_arg, np.int64),
                      str_off=np.ascontiguousarray(str_off, np.int64),
                      str_bytes=np.frombuffer(bytes(str_bytes) + b"\0", np.uint8))
        self.interned = interned

    @property
    def n_problems(self) -> int:
        return len(self.a["prob_var_off"]) - 1

    def slice(self, p0: int, p1: int) -> "WireArrays":
        """Problems [p0, p1) as a wire batch of their own, without a copy: the
        offsets are absolute (include/deppy_hip.h dp_wire), so the range's
        prob_var_off is a view into this batch's and every other array is
        shared."""
        w = WireArrays.__new__(WireArrays)
        w.a = dict(self.a)
        w.a["prob_var_off"] = self.a["prob_var_off"][p0:p1 + 1]
        w.interned = self.interned
        return w

    def struct(self) -> Wire:
        a = self.a
        # keep one extra element so empty arrays still have a valid pointer
        for k in ("var_id", "con_kind", "con_n", "con_arg"):
            if len(a[k]) == 0:
                a[k] = np.zeros(1, a[k].dtype)
        w = Wire()
        w.n_problems = len(a["prob_var_off"]) - 1
        w.prob_var_off = _p(a["prob_var_off"], c_i64p)
        w.var_id = _p(a["var_id"], c_i64p)
        w.var_con_off = _p(a["var_con_off"], c_i64p)
        w.con_kind = _p(a["con_kind"], c_i32p)
        w.con_n = _p(a["con_n"], c_i32p)
        w.con_arg_off = _p(a["con_arg_off"], c_i64p)
        w.con_arg = _p(a["con_arg"], c_i64p)
        w.n_strs = len(a["str_off"]) - 1
        w.str_off = _p(a["str_off"], c_i64p)
        w.str_bytes = ctypes.cast(a["str_bytes"].ctypes.data, ctypes.c_char_p)
        w.interned = 1 if self.interned else 0
        return w


def wire_to_numpy(w: Wire) -> dict:
    """Copy a C-owned dp_wire (e.g. from dp_gen_wire) into numpy arrays."""
    P = w.n_problems
    pvo = np.ctypeslib.as_array(w.prob_var_off, (P + 1,)).copy()
    nv = int(pvo[-1])
    vco = np.ctypeslib.as_array(w.var_con_off, (nv + 1,)).copy() if nv else np.zeros(1, np.int64)
    nc = int(vco[-1])
    cao = np.ctypeslib.as_array(w.con_arg_off, (nc + 1,)).copy() if nc else np.zeros(1, np.int64)
    na = int(cao[-1])
    so = np.ctypeslib.as_array(w.str_off, (w.n_strs + 1,)).copy()
    sb = ctypes.string_at(w.str_bytes, int(so[-1]))
    return dict(prob_var_off=pvo,
                var_id=np.ctypeslib.as_array(w.var_id, (nv,)).copy() if nv else np.zeros(0, np.int64),
                var_con_off=vco,
                con_kind=np.ctypeslib.as_array(w.con_kind, (nc,)).copy() if nc else np.zeros(0, np.int32),
                con_n=np.ctypeslib.as_array(w.con_n, (nc,)).copy() if nc else np.zeros(0, np.int32),
                con_arg_off=cao,
                con_arg=np.ctypeslib.as_array(w.con_arg, (na,)).copy() if na else np.zeros(0, np.int64),
                str_off=so, str_bytes=np.frombuffer(sb, np.uint8))


class _LoweredHandle:
    """Owns a dp_lowered; numpy views of its arrays keep it alive."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        try:
            if self.h:
                lib().dp_lowered_free(self.h)
        except Exception:
            pass


def _view(owner, ptr, n: int, ctype, dtype) -> np.ndarray:
    """Zero-copy numpy view of n elements at ptr, holding `owner` alive."""
    if n == 0:
        return np.zeros(0, dtype)
    arr = (ctype * n).from_address(ctypes.cast(ptr, ctypes.c_void_p).value)
    arr._owner = owner
    return np.frombuffer(arr, dtype)


class Lowered:
    """Result of dp_lower: numpy views of the library-owned arrays (no copy).
    relower(wire) lowers another batch into the same storage
    (dp_lower_into), invalidating the previous views' contents."""

    def __init__(self, wire: WireArrays, narrow: bool = False, pinned: bool = False, packed: bool = False,
                 p8: bool = True):
        """narrow: records that fit 16 bits in the DP_FMT_U16 form, each on a
        16-byte boundary (the staged form, DP_LOWER_NARROW); default int32
        records.  pinned: the records in page-locked memory when a GPU is
        present (DP_LOWER_PINNED; with narrow, dp_submit copies them to the
        device without staging).  packed (with narrow): the packed forms
        where they apply (DP_LOWER_PACKED: DP_FMT_P8D, DP_FMT_P16D or
        DP_FMT_P16); p8=False keeps DP_FMT_P16D (DP_LOWER_NO_P8)."""
        L = lib()
        h = ctypes.c_void_p()
        ws = wire.struct()
        self.narrow = narrow
        self._flags = (1 if narrow else 0) | (2 if pinned else 0) | (4 if packed else 0) | (0 if p8 else 8)
        if self._flags:
            h = ctypes.c_void_p(L.dp_lowered_new())
            if L.dp_lower_into(ctypes.byref(ws), self._flags, h) != 0:
                L.dp_lowered_free(h)
                raise ValueError(L.dp_last_global_error().decode())
        elif L.dp_lower(ctypes.byref(ws), ctypes.byref(h)) != 0:
            raise ValueError(L.dp_last_global_error().decode())
        self._owner = _LoweredHandle(h)
        self._fetch()

    def relower(self, wire: WireArrays) -> "Lowered":
        ws = wire.struct()
        if lib().dp_lower_into(ctypes.byref(ws), self._flags, self._owner.h) != 0:
            raise ValueError(lib().dp_last_global_error().decode())
        self._fetch()
        return self

    def _cview(self, key, ptr, n: int, ctype, dtype) -> np.ndarray:
        """_view, reused while the storage stays where it is (a serving loop
        lowers batch after batch into the same storage: no new views)."""
        addr = ctypes.cast(ptr, ctypes.c_void_p).value if n else 0
        vc = self.__dict__.setdefault("_vc", {})
        c = vc.get(key)
        if c is not None and c[0] == addr and c[1] == n:
            return c[2]
        v = _view(self._owner, ptr, n, ctype, dtype)
        vc[key] = (addr, n, v)
        return v

    def _fetch(self):
        L, h = lib(), self._owner.h
        P = L.dp_lowered_num_problems(h)
        self.n = P
        self.n_exact = int(L.dp_lowered_exact_count(h))
        self.pinned = bool(L.dp_lowered_pinned(h))
        self.rec_off = self._cview("rec_off", L.dp_lowered_rec_off(h), P + 1, ctypes.c_int64, np.int64)
        self.rec = self._cview("rec", L.dp_lowered_rec(h), int(self.rec_off[-1]), ctypes.c_int32, np.int32)
        self.ident_off = self._cview("ident_off", L.dp_lowered_ident_off(h), P + 1, ctypes.c_int64, np.int64)
        ni = int(self.ident_off[-1])
        self.ident_var = self._cview("ident_var", L.dp_lowered_ident_var(h), ni, ctypes.c_int32, np.int32)
        self.ident_con = self._cview("ident_con", L.dp_lowered_ident_con(h), ni, ctypes.c_int32, np.int32)
        err = np.zeros(max(P, 1), np.int32)
        msg = [None] * P
        m = ctypes.c_char_p()
        if L.dp_lowered_errors(h, _p(err, c_i32p)):
            for p in np.nonzero(err[:P])[0]:
                L.dp_lowered_error(h, int(p), ctypes.byref(m))
                msg[p] = m.value.decode("utf-8", "surrogateescape")
        self.err = err[:P]
        self.msg = msg

    def record(self, p: int) -> np.ndarray:
        return self.rec[self.rec_off[p]:self.rec_off[p + 1]]

    @classmethod
    def empty(cls, narrow: bool = True, pinned: bool = True, packed: bool = True, p8: bool = True) -> "Lowered":
        """An empty result for another lowering to fill (DeviceLowerer.lower)."""
        self = cls.__new__(cls)
        self.narrow = narrow
        self._flags = (1 if narrow else 0) | (2 if pinned else 0) | (4 if packed else 0) | (0 if p8 else 8)
        self._owner = _LoweredHandle(ctypes.c_void_p(lib().dp_lowered_new()))
        self.n, self.n_exact, self.pinned = 0, 0, False
        self.rec_off = self.ident_off = np.zeros(1, np.int64)
        self.rec = self.ident_var = self.ident_con = self.err = np.zeros(0, np.int32)
        self.msg = []
        return self


class HostArray:
    """n elements of page-locked host memory (dp_host_alloc) as a numpy array,
    or ordinary numpy memory when there is no device."""

    def __init__(self, n: int, dtype):
        dt = np.dtype(dtype)
        nb = max(int(n), 1) * dt.itemsize
        self._p = lib().dp_host_alloc(nb)  # NULL without a device
        if self._p:
            buf = (ctypes.c_char * nb).from_address(self._p)
            self.a = np.frombuffer(buf, dt, count=max(int(n), 1))[:int(n)]
        else:
            self.a = np.zeros(max(int(n), 1), dt)[:int(n)]

    def __del__(self):
        try:
            if self._p:
                self.a = None
                lib().dp_host_free(self._p)
                self._p = None
        except Exception:
            pass


class Wire32Arrays:
    """A dp_wire32 (include/deppy_hip.h), the compact wire: per problem the
    absolute offsets of its variables, constraints and arguments, per
    variable and constraint a 16-bit count, a constraint's kind and bound in
    one word; with at most 65,536 strings (and ids16) the string indices in
    16 bits.  In page-locked memory when a device is present, so
    dp_lower_device's copy to the device runs by DMA from where it lies."""

    ARRAYS = (("prob_var_off", np.int32), ("prob_con_off", np.int32), ("prob_arg_off", np.int32),
              ("var_id", np.int32), ("var_ncon", np.uint16), ("con_kn", np.int32), ("con_nargs", np.uint16),
              ("con_arg", np.int32))

    def __init__(self, wire: WireArrays, pinned: bool = True, ids16: bool = True):
        w = wire.a
        pvo = w["prob_var_off"]
        vco, cao = w["var_con_off"], w["con_arg_off"]
        pco = vco[pvo] if len(vco) else np.zeros(len(pvo), np.int64)
        pao = cao[pco] if len(cao) else np.zeros(len(pvo), np.int64)
        n = w["con_n"].astype(np.int64)
        src = dict(prob_var_off=pvo, prob_con_off=pco, prob_arg_off=pao, var_id=w["var_id"],
                   var_ncon=np.diff(vco) if len(vco) > 1 else np.zeros(0, np.int64),
                   con_kn=w["con_kind"].astype(np.int64) | (n << 3),
                   con_nargs=np.diff(cao) if len(cao) > 1 else np.zeros(0, np.int64),
                   con_arg=w["con_arg"])
        self.ids16 = ids16 and len(w["str_off"]) - 1 <= 65536
        if self.ids16:
            src["var_id16"], src["con_arg16"] = src.pop("var_id"), src.pop("con_arg")
        self._bufs = {}
        self.a = {}
        for k, dt in self.arrays():
            x = np.asarray(src[k])
            info = np.iinfo(dt)
            if len(x) and (x.max() > info.max or x.min() < info.min) or (k == "con_kn" and len(n) and (
                    n.max() >= 1 << 28 or n.min() < -(1 << 28))):
                raise ValueError("dp_wire32: %s does not fit %d bits" % (k, 8 * np.dtype(dt).itemsize))
            if pinned:
                b = HostArray(len(x), dt)
                b.a[:] = x
                self._bufs[k] = b
                self.a[k] = b.a
            else:
                self.a[k] = np.ascontiguousarray(x, dt)
        self.a["str_off"] = w["str_off"]
        self.a["str_bytes"] = w["str_bytes"]
        self._pad32 = np.zeros(1, np.int32)
        self._pad16 = np.zeros(1, np.uint16)

    def arrays(self):
        if not self.ids16:
            return self.ARRAYS
        wide = {"var_id": "var_id16", "con_arg": "con_arg16"}
        return tuple((wide[k], np.uint16) if k in wide else (k, dt) for k, dt in self.ARRAYS)

    @property
    def n_problems(self) -> int:
        return len(self.a["prob_var_off"]) - 1

    def nbytes(self) -> int:
        return int(sum(self.a[k].nbytes for k, _ in self.arrays()))

    def struct(self) -> Wire32:
        """The dp_wire32 over these arrays (built once: they do not move)."""
        if getattr(self, "_struct", None) is not None:
            return self._struct
        a = self.a
        w = Wire32()
        w.n_problems = len(a["prob_var_off"]) - 1
        for k, dt in self.arrays():
            if dt == np.uint16:
                setattr(w, k, _p(a[k] if len(a[k]) else self._pad16, ctypes.POINTER(ctypes.c_uint16)))
            else:
                setattr(w, k, _p(a[k] if len(a[k]) else self._pad32, c_i32p))
        w.n_strs = len(a["str_off"]) - 1
        w.str_off = _p(a["str_off"], c_i64p)
        w.str_bytes = ctypes.cast(a["str_bytes"].ctypes.data, ctypes.c_char_p)
        self._struct = w
        return w


class DeviceLowerer:
    """dp_dlower: lowering on the context's first device (dp_lower_device),
    the same records as dp_lower_into, byte for byte."""

    def __init__(self, ctx: "Context"):
        h = lib().dp_dlower_new(ctx.h)
        if not h:
            raise RuntimeError(lib().dp_last_global_error().decode())
        self.h = h
        self.ctx = ctx  # (outlives the lowering object)

    def lower(self, w32: Wire32Arrays, lw: Lowered | None = None, pinned: bool = True) -> Lowered:
        if lw is None:
            lw = Lowered.empty(pinned=pinned)
        ws = w32.struct()
        if lib().dp_lower_device(self.h, ctypes.byref(ws), lw._flags, lw._owner.h) != 0:
            raise ValueError(lib().dp_last_global_error().decode())
        lw._fetch()
        return lw

    @property
    def host_count(self) -> int:
        """Problems of the last call lowered on the host."""
        return int(lib().dp_dlower_host_count(self.h))

    def close(self):
        if self.h:
            lib().dp_dlower_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# device context and batch solve
# ---------------------------------------------------------------------------
class Context:
    def __init__(self, first_device: int = 0, n_devices: int = 1, step_budget: int = 0,
                 flags: int = 0):
        L = lib()
        o = Opts(first_device, n_devices, step_budget, flags)
        h = L.dp_create(ctypes.byref(o))
        if not h:
            raise RuntimeError("deppy_amd: no usable MI355X: " + L.dp_last_global_error().decode())
        self.h = h

    def close(self):
        if self.h:
            lib().dp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error(self) -> str:
        return lib().dp_last_error(self.h).decode()

    def lanes(self) -> int:
        """Pipeline chunk slots per device (dp_lanes): chunks a serving loop keeps in flight."""
        return int(lib().dp_lanes(self.h)) if hasattr(lib(), "dp_lanes") else 8

    def upload(self, rec_off: np.ndarray, rec: np.ndarray, trace_cap: int = 0) -> "Resident":
        return Resident(self, rec_off, rec, trace_cap)

    def solve(self, rec_off: np.ndarray, rec: np.ndarray, trace_cap: int = 0) -> dict:
        """Host records -> host results (dp_solve).  trace_cap > 0 goes through
        the device-resident form and also returns the search trace
        (dp_upload_traced): trace[P, trace_cap], trace_len[P]."""
        if trace_cap <= 0:
            rec_off = np.ascontiguousarray(rec_off, np.int64)
            rec = np.ascontiguousarray(rec if len(rec) else np.zeros(1, np.int32), np.int32)
            out = result_arrays(rec_off, rec)
            r = _result_struct(out)
            if lib().dp_solve(self.h, ctypes.byref(_batch(rec_off, rec)), ctypes.byref(r)) != 0:
                raise RuntimeError("dp_solve: " + self.error())
            n = len(rec_off) - 1
            for k in ("status", "flags", "core_len", "steps"):
                out[k] = out[k][:n]
            return out
        r = self.upload(rec_off, rec, trace_cap)
        try:
            r.run()
            out = r.download()
            out.update(r.download_trace())
            return out
        finally:
            r.free()

    def submit(self, rec_off: np.ndarray, rec: np.ndarray, out: dict | None = None) -> "Job":
        """Asynchronous host-to-host solve (dp_submit); Job.wait() -> results.
        `out` (a previous result dict of the same batch) is reused in place."""
        return Job(self, rec_off, rec, out)

    def stats(self, reset: bool = False) -> dict:
        st = Stats()
        lib().dp_get_stats(self.h, ctypes.byref(st), 1 if reset else 0)
        return _stats_dict(st)

    def devices(self) -> int:
        """Logical devices of the context (dp_num_devices)."""
        return int(lib().dp_num_devices(self.h))

    def device_stats(self, device: int, reset: bool = False) -> dict:
        """dp_get_device_stats: the share of the pipeline one logical device ran."""
        st = Stats()
        if lib().dp_get_device_stats(self.h, device, ctypes.byref(st), 1 if reset else 0) != 0:
            raise ValueError("dp_get_device_stats: no device %d" % device)
        return _stats_dict(st)

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_double()
        lib().dp_last_kernel_ms(self.h, ctypes.byref(ms))
        return ms.value


def _batch(rec_off, rec):
    b = Batch()
    b.n_problems = len(rec_off) - 1
    b.rec_off = _p(rec_off, c_i64p)
    b.rec = _p(rec, c_i32p)
    return b


def result_arrays(rec_off, rec) -> dict:
    """Caller-allocated dp_result arrays for a batch (dp_result_layout),
    their pages touched here: np.zeros maps large arrays lazily, and the
    pipeline's scatter would otherwise take the page faults of a buffer's
    first use (config 6: 0.23 instead of 0.055 ms per 10k results)."""
    rec_off = np.ascontiguousarray(rec_off, np.int64)
    n = len(rec_off) - 1
    inst_off = np.zeros(n + 1, np.int64)
    core_off = np.zeros(n + 1, np.int64)
    lib().dp_result_layout(ctypes.byref(_batch(rec_off, rec)), _p(inst_off, c_i64p), _p(core_off, c_i64p))

    def zeros(m, dt):
        a = np.empty(m, dt)
        a.fill(0)
        return a
    return dict(status=zeros(max(n, 1), np.int8), flags=zeros(max(n, 1), np.int32),
                installed=zeros(max(1, int(inst_off[-1])), np.uint32), inst_off=inst_off,
                core=zeros(max(1, int(core_off[-1])), np.int32), core_off=core_off,
                core_len=zeros(max(n, 1), np.int32), steps=zeros(max(n, 1), np.int64))


def _result_struct(out: dict) -> Result:
    return Result(_p(out["status"], c_i8p), _p(out["flags"], c_i32p), _p(out["installed"], c_u32p),
                  _p(out["inst_off"], c_i64p), _p(out["core"], c_i32p), _p(out["core_off"], c_i64p),
                  _p(out["core_len"], c_i32p), _p(out["steps"], c_i64p))


class Job:
    """A host-to-host solve in flight (dp_submit); wait() -> result dict."""

    def __init__(self, ctx: Context, rec_off, rec, out: dict | None = None):
        self.ctx = ctx
        rec_off = np.ascontiguousarray(rec_off, np.int64)
        rec = np.ascontiguousarray(rec if len(rec) else np.zeros(1, np.int32), np.int32)
        self.n = len(rec_off) - 1
        self.out = out if out is not None else result_arrays(rec_off, rec)
        self._res = _result_struct(self.out)
        # the device's worker thread reads the batch after dp_submit returns:
        # the arrays (possibly converted copies) live as long as the job
        self._batch_arrays = (rec_off, rec)
        h = ctypes.c_void_p()
        if lib().dp_submit(ctx.h, ctypes.byref(_batch(rec_off, rec)), ctypes.byref(self._res),
                           ctypes.byref(h)) != 0:
            raise RuntimeError("dp_submit: " + ctx.error())
        self.h = h

    def wait(self) -> dict:
        h, self.h = self.h, None
        if h is None:
            raise RuntimeError("dp_job_wait: job already waited")
        rc = lib().dp_job_wait(self.ctx.h, h)
        self._batch_arrays = None
        if rc != 0:
            raise RuntimeError("dp_job_wait: " + self.ctx.error())
        out = dict(self.out)
        for k in ("status", "flags", "core_len", "steps"):
            out[k] = out[k][:self.n]
        return out


class Resident:
    """A batch resident in HBM (dp_upload); run() solves it in place."""

    def __init__(self, ctx: Context, rec_off, rec, trace_cap: int = 0):
        self.ctx = ctx
        self.trace_cap = trace_cap
        self.rec_off = np.ascontiguousarray(rec_off, np.int64)
        self.rec = np.ascontiguousarray(rec if len(rec) else np.zeros(1, np.int32), np.int32)
        n = len(self.rec_off) - 1
        self.n = n
        b = _batch(self.rec_off, self.rec)
        self.inst_off = np.zeros(n + 1, np.int64)
        self.core_off = np.zeros(n + 1, np.int64)
        lib().dp_result_layout(ctypes.byref(b), _p(self.inst_off, c_i64p), _p(self.core_off, c_i64p))
        h = ctypes.c_void_p()
        if lib().dp_upload_traced(ctx.h, ctypes.byref(b), trace_cap, ctypes.byref(h)) != 0:
            raise RuntimeError("dp_upload: " + ctx.error())
        self.h = h

    def run(self):
        if lib().dp_run(self.ctx.h, self.h) != 0:
            raise RuntimeError("dp_run: " + self.ctx.error())

    def launch(self):
        """Enqueue a solve of the batch and return (dp_launch)."""
        if lib().dp_launch(self.ctx.h, self.h) != 0:
            raise RuntimeError("dp_launch: " + self.ctx.error())

    def wait(self):
        """Block until the last launch finished (dp_wait)."""
        if lib().dp_wait(self.ctx.h, self.h) != 0:
            raise RuntimeError("dp_wait: " + self.ctx.error())

    def download(self) -> dict:
        n = self.n
        out = result_arrays(self.rec_off, self.rec)
        r = _result_struct(out)
        if lib().dp_download(self.ctx.h, self.h, ctypes.byref(r)) != 0:
            raise RuntimeError("dp_download: " + self.ctx.error())
        for k in ("status", "flags", "core_len", "steps"):
            out[k] = out[k][:n]
        return out

    def download_trace(self) -> dict:
        n = self.n
        tr = np.zeros((max(n, 1), max(self.trace_cap, 1)), np.int32)
        tl = np.zeros(max(n, 1), np.int32)
        if lib().dp_download_trace(self.ctx.h, self.h, _p(tr, c_i32p), _p(tl, c_i32p)) != 0:
            raise RuntimeError("dp_download_trace: " + self.ctx.error())
        return dict(trace=tr[:n], trace_len=tl[:n])

    def free(self):
        if self.h:
            lib().dp_resident_free(self.ctx.h, self.h)
            self.h = None


def device_bytes(rec_off, rec, flags: int = 0) -> tuple[int, int]:
    """(record bytes, image bytes) of a batch in its device form (dp_device_bytes)."""
    rec_off = np.ascontiguousarray(rec_off, np.int64)
    rec = np.ascontiguousarray(rec if len(rec) else np.zeros(1, np.int32), np.int32)
    rb, ib = ctypes.c_int64(), ctypes.c_int64()
    if lib().dp_device_bytes(ctypes.byref(_batch(rec_off, rec)), flags, ctypes.byref(rb), ctypes.byref(ib)) != 0:
        raise RuntimeError("dp_device_bytes failed")
    return rb.value, ib.value


def plan_placements(rec_off, rec, flags: int = 0) -> np.ndarray:
    """Per-problem placement dp_submit plans for a batch cut as one chunk
    (dp_plan_placements: an index into PLACES, or -1 malformed / -2 too large)."""
    rec_off = np.ascontiguousarray(rec_off, np.int64)
    rec = np.ascontiguousarray(rec if len(rec) else np.zeros(1, np.int32), np.int32)
    place = np.zeros(max(len(rec_off) - 1, 1), np.int8)
    if lib().dp_plan_placements(ctypes.byref(_batch(rec_off, rec)), flags, _p(place, c_i8p)) != 0:
        raise RuntimeError("dp_plan_placements failed")
    return place[:len(rec_off) - 1]


def plan_order(rec_off, rec, flags: int = 0):
    """(order, launch_first): the workgroup order dp_submit plans for a batch
    cut as one chunk (dp_plan_order)."""
    rec_off = np.ascontiguousarray(rec_off, np.int64)
    rec = np.ascontiguousarray(rec if len(rec) else np.zeros(1, np.int32), np.int32)
    order = np.zeros(max(len(rec_off) - 1, 1), np.int32)
    first = np.zeros(32, np.int32)
    nl = lib().dp_plan_order(ctypes.byref(_batch(rec_off, rec)), flags, _p(order, c_i32p), _p(first, c_i32p))
    if nl < 0:
        raise RuntimeError("dp_plan_order failed")
    return order, first[:nl]


def stage_roundtrip(rec_off, rec, flags: int = 0, chunk_problems: int = 0, chunk_bytes: int = 0):
    """Host-only: stage a batch in chunks as dp_submit does and widen it back
    (dp_stage_roundtrip) -> (records, first problem of each chunk)."""
    rec_off = np.ascontiguousarray(rec_off, np.int64)
    rec = np.ascontiguousarray(rec if len(rec) else np.zeros(1, np.int32), np.int32)
    out = np.zeros_like(rec)
    firsts = np.zeros(max(len(rec_off), 1), np.int32)
    k = lib().dp_stage_roundtrip(ctypes.byref(_batch(rec_off, rec)), flags, chunk_problems, chunk_bytes,
                                 _p(out, c_i32p), _p(firsts, c_i32p), len(firsts))
    if k < 0:
        raise ValueError("dp_stage_roundtrip: malformed record")
    return out, firsts[:k]


def stitch_selftest(rec_off, rec, chunk_problems: int) -> dict:
    """Host-only: synthetic per-problem results scattered chunk by chunk
    (dp_stitch_selftest)."""
    rec_off = np.ascontiguousarray(rec_off, np.int64)
    rec = np.ascontiguousarray(rec, np.int32)
    out = result_arrays(rec_off, rec)
    out["installed"][:] = 0xdeadbeef
    r = _result_struct(out)
    if lib().dp_stitch_selftest(ctypes.byref(_batch(rec_off, rec)), chunk_problems, ctypes.byref(r)) < 0:
        raise ValueError("dp_stitch_selftest failed")
    return out


def partition(rec_off, nd: int) -> np.ndarray:
    rec_off = np.ascontiguousarray(rec_off, np.int64)
    cut = np.zeros(nd + 1, np.int32)
    if lib().dp_partition(_p(rec_off, c_i64p), len(rec_off) - 1, nd, _p(cut, c_i32p)) != 0:
        raise ValueError("dp_partition failed")
    return cut


def generate(config: int, n: int, seed: int) -> dict:
    """Synthetic catalogs (dp_gen_catalogs) as numpy wire arrays."""
    L = lib()
    g = L.dp_gen_catalogs(config, n, seed)
    if not g:
        raise ValueError(L.dp_last_global_error().decode())
    try:
        return wire_to_numpy(L.dp_gen_wire(g).contents)
    finally:
        L.dp_gen_free(g)


def trace_events(res: dict, p: int) -> list:
    """The search-trace events of problem p: [(guessed variables, identities)]."""
    t = res["trace"][p][:int(res["trace_len"][p])]
    ev, i = [], 0
    while i < len(t):
        n = int(t[i])
        vs = [int(x) for x in t[i + 1:i + 1 + n]]
        i += 1 + n
        m = int(t[i])
        ev.append((vs, [int(x) for x in t[i + 1:i + 1 + m]]))
        i += 1 + m
    return ev


def installed_list(res: dict, p: int, nv: int) -> list[int]:
    base = int(res["inst_off"][p])
    words = res["installed"][base:base + (nv + 31) // 32]
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:nv]
    return [int(i) for i in np.flatnonzero(bits)]


def core_list(res: dict, p: int) -> list[int]:
    base = int(res["core_off"][p])
    return [int(x) for x in res["core"][base:base + int(res["core_len"][p])]]
