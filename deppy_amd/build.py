"""Builds libdeppy_hip.so in-tree with hipcc for gfx950 (no JIT cache, so the
.so travels with the repo snapshot to the GPU box)."""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libdeppy_hip.so")
OBJ = os.path.join(HERE, "_obj")
# diagnostic variant (phase stamps); never loaded by the product path
STAMPS_LIB = os.path.join(HERE, "libdeppy_hip_stamps.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
SOURCES = ["solve_lds.hip", "solve_lds_dense.hip", "solve_split.hip", "solve_split4.hip", "solve_ldsg.hip", "solve_hbm.hip", "watch_build.hip", "lower_device.hip", "solve_launch.cpp", "runtime.cpp",
           "lower.cpp", "gen.cpp"]
FLAGS = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
         "--offload-arch=" + ARCH, "-I" + os.path.join(HERE, "..", "include")]


def _headers() -> list[str]:
    hs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h")))
    return hs + [os.path.join(HERE, "..", "include", "deppy_hip.h")]


def sources_digest(extra: list[str] | None = None) -> str:
    """sha256 (first 16 hex digits) of every source and header the library is
    compiled from and of the compile flags.  The library carries it
    (dp_build_info), and the binding refuses a product library whose digest
    is not the tree's: the .so that runs is the one these sources make."""
    h = hashlib.sha256()
    for f in [os.path.join(CSRC, x) for x in SOURCES] + _headers():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    h.update(" ".join(FLAGS[:-1] + (extra or [])).encode())  # (the include path is the tree's own)
    return h.hexdigest()[:16]


def _file_digest(paths: list[str], extra: list[str] | None) -> str:
    h = hashlib.sha256()
    for f in paths:
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    h.update(" ".join(FLAGS[:-1] + (extra or [])).encode())
    return h.hexdigest()[:16]


def _needs(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, extra: list[str] | None = None, stamps: bool = False,
          tag: str = "") -> str:
    global OBJ, LIB
    if extra and not stamps and not tag:
        # the product library is the tree's sources with the tree's flags (the
        # binding checks its digest); other flags make a tagged variant
        raise ValueError("build(extra=...) makes a measurement variant: give it a tag")
    if stamps:
        extra = (extra or []) + ["-DDP_STAMPS"]
        obj, lib = OBJ + "_stamps" + tag, STAMPS_LIB.replace(".so", tag + ".so")
    else:  # a tagged release variant (measurement only) never replaces the product library
        obj, lib = OBJ + tag, LIB.replace(".so", tag + ".so")
    return _build(verbose, extra, obj, lib)


def _build(verbose, extra, OBJ, LIB) -> str:
    os.makedirs(OBJ, exist_ok=True)
    headers = _headers()
    digest = sources_digest(extra)
    stamp = os.path.join(OBJ, "digest")
    # objects follow their sources' mtimes; a digest change (sources or
    # flags) relinks, so the embedded digest is always the tree's
    stale = not os.path.exists(stamp) or open(stamp).read().strip() != digest
    jobs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src + ".o")
        # an object is rebuilt when its inputs' contents differ from the ones
        # it was compiled from (not only when they are newer)
        od = _file_digest([s] + headers, extra)
        dfile = o + ".digest"
        same = os.path.exists(dfile) and open(dfile).read().strip() == od
        if not same or _needs(o, [s] + headers) or extra:
            lang = ["-x", "hip"] if src.endswith(".hip") or src in ("runtime.cpp", "solve_launch.cpp") else []
            jobs.append(([HIPCC] + FLAGS + (extra or []) + lang + ["-c", s, "-o", o], dfile, od))
    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    def compile_one(job):
        cmd, dfile, od = job
        if os.path.exists(dfile):
            os.remove(dfile)  # (a failed or interrupted compile leaves no digest)
        run(cmd)
        with open(dfile, "w") as f:
            f.write(od + "\n")
    with ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(compile_one, jobs))
    objs = [os.path.join(OBJ, s + ".o") for s in SOURCES]
    if stale or _needs(LIB, objs) or jobs:
        # the digest, compiled into the library (dp_build_info)
        info = os.path.join(OBJ, "build_info.cpp")
        with open(info, "w") as f:
            f.write('extern "C" const char* dp_build_info(void) { return "sources=%s arch=%s"; }\n' % (digest, ARCH))
        run([HIPCC] + FLAGS + ["-c", info, "-o", info + ".o"])
        run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs + [info + ".o", "-lpthread"])
    with open(stamp, "w") as f:
        f.write(digest + "\n")
    return LIB


if __name__ == "__main__":
    args = sys.argv[1:]
    stamps = "--stamps" in args
    tag = next((a.split("=", 1)[1] for a in args if a.startswith("--tag=")), "")
    args = [a for a in args if a != "--stamps" and not a.startswith("--tag=")]
    build(verbose=True, extra=args or None, stamps=stamps, tag=tag)
