"""ctypes wrapper of the CPU restatement (libsat_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package (deppy_amd/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libsat_oracle.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_i8p = np.ctypeslib.ndpointer(dtype=np.int8, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = _bind(ctypes.CDLL(_LIB))
    return _lib


_twl = None


def twl_lib():
    """The restatement with the kernel's two-watched-literal lists (make's
    libsat_oracle_twl.so, -DORACLE_TWL), plus its round counters."""
    global _twl
    if _twl is None:
        path = os.path.join(_HERE, "libsat_oracle_twl.so")
        if not os.path.exists(path):
            build()
        L = _bind(ctypes.CDLL(path))
        L.oracle_twl_stats.argtypes = [np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS"), ctypes.c_int]
        _twl = L
    return _twl


def _bind(L):
    L.oracle_solve.argtypes = [_i32p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32), _u32p,
                               _i32p, ctypes.POINTER(ctypes.c_int32),
                               ctypes.POINTER(ctypes.c_int64)]
    L.oracle_solve.restype = ctypes.c_int
    L.oracle_solve_batch.argtypes = [ctypes.c_int32, _i64p, _i32p, ctypes.c_int64,
                                     ctypes.c_int32, _i8p, _i32p, _u32p, _i64p, _i32p,
                                     _i64p, _i32p, _i64p]
    L.oracle_solve_batch_traced.argtypes = [ctypes.c_int32, _i64p, _i32p, ctypes.c_int64,
                                            ctypes.c_int32, _i8p, _i32p, _u32p, _i64p, _i32p,
                                            _i64p, _i32p, _i64p, _i32p, ctypes.c_int32, _i32p]
    L.oracle_search_scripted.argtypes = [_i32p, _i32p, ctypes.c_int32, _i32p, ctypes.c_int32,
                                         ctypes.POINTER(ctypes.c_int32), _i32p,
                                         ctypes.POINTER(ctypes.c_int32),
                                         ctypes.POINTER(ctypes.c_int32)]
    L.oracle_refute.argtypes = [_i32p, ctypes.c_void_p, ctypes.c_int64]
    L.oracle_refute.restype = ctypes.c_int
    L.oracle_check_model.argtypes = [_i32p, _u32p]
    L.oracle_check_model.restype = ctypes.c_int
    return L


def nv_of(rec) -> int:
    return int(rec[1])


def nid_of(rec) -> int:
    return int(rec[6])


def solve(rec: np.ndarray, budget: int = 0):
    """-> (status, flags, installed_vars(list), core(list of identity ids), steps)"""
    rec = np.ascontiguousarray(rec, dtype=np.int32)
    nv, nid = nv_of(rec), nid_of(rec)
    inst = np.zeros(max(1, (nv + 31) // 32), dtype=np.uint32)
    core = np.zeros(max(1, nid), dtype=np.int32)
    flags, clen, steps = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
    st = lib().oracle_solve(rec, budget, ctypes.byref(flags), inst, core, ctypes.byref(clen),
                            ctypes.byref(steps))
    installed = [v for v in range(nv) if (int(inst[v >> 5]) >> (v & 31)) & 1]
    return st, flags.value, installed, list(core[:clen.value]), steps.value


def solve_batch(rec_off: np.ndarray, rec: np.ndarray, budget: int = 0, nthreads: int = 1,
                trace_cap: int = 0, L=None):
    """Batch solve; returns dict of arrays (same layout as dp_result).  With
    trace_cap > 0 also the search trace: trace[P, trace_cap], trace_len[P]."""
    rec_off = np.ascontiguousarray(rec_off, dtype=np.int64)
    rec = np.ascontiguousarray(rec, dtype=np.int32)
    n = len(rec_off) - 1
    nvs = rec[rec_off[:-1] + 1].astype(np.int64)  # (headers are int32 in either record form)
    nids = rec[rec_off[:-1] + 6].astype(np.int64)
    inst_off = np.zeros(n + 1, np.int64)
    inst_off[1:] = np.cumsum((nvs + 31) // 32)
    core_off = np.zeros(n + 1, np.int64)
    core_off[1:] = np.cumsum(nids)
    out = dict(
        status=np.zeros(n, np.int8), flags=np.zeros(n, np.int32),
        installed=np.zeros(max(1, int(inst_off[-1])), np.uint32), inst_off=inst_off,
        core=np.zeros(max(1, int(core_off[-1])), np.int32), core_off=core_off,
        core_len=np.zeros(n, np.int32), steps=np.zeros(n, np.int64))
    if trace_cap > 0:
        out["trace"] = np.zeros((n, trace_cap), np.int32)
        out["trace_len"] = np.zeros(n, np.int32)
        (L or lib()).oracle_solve_batch_traced(n, rec_off, rec, budget, nthreads, out["status"],
                                        out["flags"], out["installed"], inst_off, out["core"],
                                        core_off, out["core_len"], out["steps"], out["trace"],
                                        trace_cap, out["trace_len"])
        return out
    (L or lib()).oracle_solve_batch(n, rec_off, rec, budget, nthreads, out["status"], out["flags"],
                             out["installed"], inst_off, out["core"], core_off, out["core_len"],
                             out["steps"])
    return out


def search_scripted(rec, test_returns, untest_returns):
    rec = np.ascontiguousarray(rec, dtype=np.int32)
    tr = np.ascontiguousarray(np.array(list(test_returns) or [0], dtype=np.int32))
    ur = np.ascontiguousarray(np.array(list(untest_returns) or [0], dtype=np.int32))
    res, nl, depth = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    lits = np.zeros(max(1, nv_of(rec)), dtype=np.int32)
    lib().oracle_search_scripted(rec, tr, len(test_returns), ur, len(untest_returns),
                                 ctypes.byref(res), lits, ctypes.byref(nl), ctypes.byref(depth))
    return res.value, list(lits[:nl.value]), depth.value


def refute(rec, enabled_idents, budget: int = 0) -> int:
    """Complete check of the rows of `enabled_idents` alone: -1 UNSAT, 1 SAT, 0 budget."""
    rec = np.ascontiguousarray(rec, dtype=np.int32)
    en = np.zeros(max(1, nid_of(rec)), dtype=np.uint8)
    for i in enabled_idents:
        en[i] = 1
    return lib().oracle_refute(rec, en.ctypes.data_as(ctypes.c_void_p), budget)


def check_model(rec, installed_words) -> int:
    """-1 if the installed bitmap satisfies every row of rec, else a violated row."""
    rec = np.ascontiguousarray(rec, dtype=np.int32)
    w = np.ascontiguousarray(installed_words, dtype=np.uint32)
    if len(w) == 0:
        w = np.zeros(1, np.uint32)
    return lib().oracle_check_model(rec, w)
