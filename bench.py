"""Benchmark: batched pkg/sat resolution on MI355X, host memory to host memory.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
                    [--scaling weak|strong]

The reference's Solve is a host-memory-to-host-memory call
(pkg/sat/solve.go:53-119).  Its benchmark times NewSolver(WithInput(...)) and
Solve together (pkg/sat/bench_test.go:66-77), lowering included: that is the
`end_to_end` figure below.  `value` times the leg BASELINE.md §3 defines for
both the GPU and the CPU baseline: lowered records in host memory ->
dp_submit (plan, H2D, solve, results into mapped host memory) -> results in
host memory (dp_job_wait), for one batch of BASELINE config 2 by default: 10,000 synthetic operator catalogs (~200 bundle entities,
Dependency + Conflict + AtMost; SURVEY.md §8(d) generator).  `--depth` jobs
are in flight, as a serving loop keeps them (default: enough to give each of the
pipeline's 8 chunk slots a chunk, 8 for a one-chunk batch): step i is submitted
before step i-depth is collected.  Every step resolves its whole batch, and every
result lands in host memory.

`value` = resolutions/s over all ranks, host to host.  Secondary figures:
`kernel_only` (the batch resident in HBM, relaunched: the rate the solve
kernel alone sustains), `host_lowering_res_per_s` (wire format -> records,
dp_lower, not in `value`), `end_to_end` (wire format -> lowering -> solve ->
results, what BenchmarkSolve times, beside lowering + the oracle on the same
cores), `latency` (one catalog alone, host to host, beside one CPU thread of
the oracle).

Multi-GPU: one process per GPU (torchrun); without WORLD_SIZE and --gpus N>1
this script relaunches itself under torch.distributed.run before touching any
GPU.  Problems are independent: no data-path collective;
torch.distributed carries only the barrier and the max-over-ranks of the
timing.  --scaling weak (default): every rank solves its own batch.
--scaling strong: the config's total (config 3: 1,000,000 catalogs) is split
across the ranks.  The topology the cgo shim ships is one process driving
every GPU (dp_create(n_devices=N)): `--inproc` measures that
instead (one process, N devices, N x the per-GPU batch), and a torchrun run
with N > 1 ranks also measures it after its own timed region (rank 0 alone
over all N GPUs while the other ranks wait), as `inproc` in the line, with the
chunks each device's submitting thread ran.

`roofline.achieved` = algorithmic bytes of a chunk (staged records + outputs,
DESIGN.md §4.2) / the chunk's solve-kernel device time (HIP events on its
stream, dp_get_stats), averaged over the timed region.  `cpu_baseline` = the
CPU restatement (oracle/, "port") on this process's CPU share (cgroup quota),
one solver per core, on the same batch repeated for a bounded time.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "resolutions/sec (node) on synthetic catalogs at 1/2/4/8 GPUs; BCP HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
PCIE_PEAK_GBS = 64.0   # PCIe Gen5 x16, one direction
LANES = 8  # chunk slots per device; replaced by the context's own count (dp_lanes) once it exists

# BASELINE.json configs as bench workloads: (catalogs per GPU, strong-scaling
# total, description)
WORKLOADS = {
    2: (10000, 80000, "config2: %d synthetic operator catalogs per step (P=40 packages, ~240 variables; "
                      "Dependency+Conflict+AtMost), one wavefront per catalog"),
    3: (125000, 1000000, "config3: %d small catalogs per step (P~U{4..12}, ~20-70 variables; 1M over the "
                         "node by host partition), one wavefront per catalog"),
    4: (256, 2048, "config4: %d OLM-scale catalogs per step (P=5000, ~55k variables, deep dependency "
                   "chains), one 8-wave workgroup per catalog"),
    5: (10000, 80000, "config5: %d mixed-size catalogs per step (P~U{4..400}, 50%% with injected "
                      "infeasibility), UNSAT-heavy"),
    6: (10000, 80000, "config6: %d problems per step shaped like the reference's BenchmarkInput "
                      "(pkg/sat/bench_test.go:10-64: 256 variables, 10%% Mandatory, 15%% one Dependency "
                      "of 1-5, 5%% 1-2 Conflicts; SplitMix64 draws, not Go's math/rand)"),
}


def cpu_share() -> dict:
    """Cores this process may use: the cgroup cpu.max quota when set (the GPU
    box gives each GPU 16), else the affinity mask."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(float(q) / float(p)))
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota": quota,
            "cores": min(aff, quota) if quota else aff}


def maybe_relaunch(args) -> None:
    """--gpus N > 1 without torchrun: run this script under
    torch.distributed.run (a child process, started before any GPU call)."""
    if args.gpus <= 1 or args.inproc or "WORLD_SIZE" in os.environ:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.exit(subprocess.call(cmd, env=env))


FORMS = {0: "I32", 1: "U16", 3: "P16", 4: "I32W", 5: "P16D", 6: "P8D"}


def record_forms(lw) -> dict:
    """Records per form (include/deppy_hip.h DP_H_FMT) of a lowered batch."""
    if lw.n == 0:
        return {}
    f, c = np.unique(lw.rec[lw.rec_off[:-1] + 13], return_counts=True)
    return {FORMS.get(int(a), str(int(a))): int(b) for a, b in zip(f, c)}


def end_to_end(ctx, wa, n, steps, depth=2):
    """Wire format -> results, what the reference's BenchmarkSolve times per
    problem (NewSolver(WithInput(...)) + Solve, pkg/sat/bench_test.go:66-77):
    each step lowers the batch (dp_lower_into into page-locked packed
    records, the host pool) and submits it; `depth` batches in flight, so the
    GPU solves batch i while the host lowers batch i+1."""
    from deppy_amd import _lib
    lws = [_lib.Lowered(wa, narrow=True, pinned=True, packed=True) for _ in range(depth)]
    outs = [_lib.result_arrays(x.rec_off, x.rec) for x in lws]

    def run(k):
        jobs = []
        for i in range(k):
            j = i % depth
            if len(jobs) == depth:
                jobs.pop(0).wait()
            lws[j].relower(wa)
            jobs.append(ctx.submit(lws[j].rec_off, lws[j].rec, outs[j]))
        for job in jobs:
            job.wait()

    run(depth)
    t0 = time.perf_counter()
    run(steps)
    return n * steps / (time.perf_counter() - t0)


def end_to_end_device(ctx, wa, lw_host, n, steps, depth=2):
    """end_to_end with the lowering on the GPU (dp_lower_device): the 32-bit
    wire in page-locked memory crosses PCIe, one wavefront per problem lowers
    it (lower_device.hip) into records that come back to page-locked host
    memory byte-identical to dp_lower_into's, and they are submitted as in
    end_to_end; `depth` batches in flight."""
    from deppy_amd import _lib
    dl = _lib.DeviceLowerer(ctx)
    w32 = _lib.Wire32Arrays(wa)
    lws = [dl.lower(w32, _lib.Lowered.empty()) for _ in range(depth)]
    same = bool(np.array_equal(lws[0].rec_off, lw_host.rec_off) and np.array_equal(lws[0].rec, lw_host.rec)
                and np.array_equal(lws[0].ident_var, lw_host.ident_var)
                and np.array_equal(lws[0].ident_con, lw_host.ident_con))
    outs = [_lib.result_arrays(x.rec_off, x.rec) for x in lws]
    t0 = time.perf_counter()
    for _ in range(3):
        dl.lower(w32, lws[0])
    t_lower = (time.perf_counter() - t0) / 3

    def run(k):
        jobs = []
        for i in range(k):
            j = i % depth
            if len(jobs) == depth:
                jobs.pop(0).wait()
            dl.lower(w32, lws[j])
            jobs.append(ctx.submit(lws[j].rec_off, lws[j].rec, outs[j]))
        for job in jobs:
            job.wait()

    run(depth)
    t0 = time.perf_counter()
    run(steps)
    rate = n * steps / (time.perf_counter() - t0)
    out = {"res_per_s": round(rate, 1), "steps": steps,
           "lowering_res_per_s": round(n / t_lower, 1), "lowering_ms": round(t_lower * 1e3, 3),
           "host_lowered_problems": dl.host_count, "wire_bytes": w32.nbytes(),
           "records_equal_host_lowering": same,
           "note": "wire (dp_wire32, page-locked) -> dp_lower_device (one wavefront per problem, "
                   "lower_device.hip; records back in page-locked host memory, byte-identical to "
                   "dp_lower_into) -> dp_submit/dp_job_wait -> results, 2 batches in flight; not value"}
    dl.close()
    return out


def solve_batch_api_device(ctx, wa, n, steps):
    """solve_batch_api from the compact wire: deppy_amd.sat.solve_wire on a
    _lib.Wire32Arrays lowers on the GPU (dp_lower_device), then dp_solve;
    one batch at a time."""
    from deppy_amd import _lib, sat
    w32 = _lib.Wire32Arrays(wa)
    sat.solve_wire(w32, ctx)
    t0 = time.perf_counter()
    for _ in range(steps):
        sat.solve_wire(w32, ctx)
    return n * steps / (time.perf_counter() - t0)


def solve_batch_api(ctx, wa, n, steps):
    """The shipped API path, one batch at a time: deppy_amd.sat.solve_wire (the
    wire -> results half of SolveBatch, what the cgo shim does): dp_lower_into
    NARROW|PACKED|PINNED into reused storage, then dp_solve on the batch as it
    lies.  No batches overlap (a caller waiting on each SolveBatch)."""
    from deppy_amd import sat
    sat.solve_wire(wa, ctx)
    t0 = time.perf_counter()
    for _ in range(steps):
        sat.solve_wire(wa, ctx)
    return n * steps / (time.perf_counter() - t0)


# Issue model of one CU (MI355X_MICROARCH.md): 4 SIMD-32 vector units, each
# issuing a wave64 VALU instruction over 2 cycles, and one scalar unit (one
# SALU instruction per cycle per CU); 256 CUs at 2.4 GHz.
CUS, CLOCK_HZ = 256, 2.4e9
VALU_PEAK = CUS * 4 * CLOCK_HZ / 2   # wave64 VALU instructions / s
SALU_PEAK = CUS * CLOCK_HZ           # SALU instructions / s


def issue_roofline(sq_json, config, res_per_s):
    """Instructions per resolution of the one-wavefront kernel (a wave per
    catalog; SQ counters of the same build, scripts/pmc_sq_r02.sh) times the
    kernel-only rate, against the VALU and SALU issue peaks."""
    if not sq_json or not os.path.exists(sq_json) or not res_per_s:
        return None
    from deppy_amd import _lib
    with open(sq_json) as f:
        j = json.load(f)
    if j.get("build") != _lib.build_info():
        # counters of another build: not this kernel's issue rate
        return {"stale": True, "source": os.path.relpath(sq_json, ROOT), "counters_build": j.get("build"),
                "note": "the SQ counters on file are not this library's (build digest differs): not reported"}
    d = j.get(str(config))
    if not d:
        return None
    pw = d["per_wave"]
    valu, salu = pw["SQ_INSTS_VALU"], pw["SQ_INSTS_SALU"]
    return {"valu_per_resolution": round(valu, 1), "salu_per_resolution": round(salu, 1),
            "lds_per_resolution": round(pw["SQ_INSTS_LDS"], 1),
            "all_per_resolution": round(sum(pw.values()), 1),
            "valu_frac": round(valu * res_per_s / VALU_PEAK, 4),
            "salu_frac": round(salu * res_per_s / SALU_PEAK, 4),
            "wave_issuing_frac": d.get("active_frac"), "wave_waiting_frac": d.get("wait_any_frac"),
            "source": os.path.relpath(sq_json, ROOT),
            "note": "kernel_only res/s x instructions per catalog (one wavefront each) / the chip's issue peak: "
                    "VALU %.3g/s (4 SIMD-32 per CU, a wave64 instruction per 2 cycles), SALU %.3g/s (one "
                    "scalar unit per CU). Both well below 1 with the waves waiting most of their cycles: the "
                    "kernel is bound by each wave's dependent LDS chain (latency), not by issue or HBM"
                    % (VALU_PEAK, SALU_PEAK)}


def cpu_end_to_end(wa, lw32, n, threads, seconds):
    """The same on the CPU: lowering to int32 records + the oracle's solve, one
    solver thread per core, for a bounded time."""
    from oracle import oracle
    reps, t0 = 0, time.perf_counter()
    while reps < 1 or time.perf_counter() - t0 < seconds:
        lw32.relower(wa)
        oracle.solve_batch(lw32.rec_off, lw32.rec, 0, threads)
        reps += 1
    return reps * n / (time.perf_counter() - t0)


def lowered_config(config, n, seed, form="packed"):
    """The batch lowered twice: in the packed 16-bit form into page-locked
    memory (dp_lower_into DP_LOWER_NARROW | DP_LOWER_PACKED | DP_LOWER_PINNED,
    as a serving loop keeps its lowering storage; what the GPU path is given)
    and as int32 records (what the CPU baseline is given).  Also the steady-state lowering rate
    (dp_lower_into reusing its storage, the wire format -> records)."""
    from deppy_amd import _lib
    w = _lib.generate(config, n, seed)
    wa = _lib.WireArrays(**{k: w[k] for k in (
        "prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off", "con_arg",
        "str_off")}, str_bytes=w["str_bytes"].tobytes())
    lw32 = _lib.Lowered(wa)
    lw = _lib.Lowered(wa, narrow=form != "i32", pinned=True, packed=form in ("packed", "p16d"), p8=form != "p16d")
    reps, t0 = 0, time.perf_counter()
    while reps < 3 or time.perf_counter() - t0 < 1.0:
        lw.relower(wa)
        reps += 1
    t_lower = (time.perf_counter() - t0) / reps
    return lw, lw32, t_lower, wa


def inproc_leg(config, n, nd, seed, steps, warmup, form):
    """The one-process topology (the cgo shim's): dp_create(n_devices=nd)
    over GPUs 0..nd-1, one batch of nd * n catalogs per step (n per device,
    as each rank of the torchrun run solves n), host to host with a job per
    chunk slot in flight.  Returns the rate and the chunks each device's
    submitting thread ran."""
    from deppy_amd import _lib
    lw, _, _, _ = lowered_config(config, n * nd, seed, form)
    ctx = _lib.Context(0, nd)
    try:
        ctx.stats(reset=True)
        ctx.submit(lw.rec_off, lw.rec).wait()
        depth = max(1, ctx.lanes() * nd // max(1, ctx.stats(reset=True)["chunks"]))
        outs = [_lib.result_arrays(lw.rec_off, lw.rec) for _ in range(depth)]

        def run(k):
            jobs = []
            for i in range(k):
                if len(jobs) == depth:
                    jobs.pop(0).wait()
                jobs.append(ctx.submit(lw.rec_off, lw.rec, outs[i % depth]))
            for j in jobs:
                j.wait()

        run(max(warmup, 1))
        ctx.stats(reset=True)
        t0 = time.perf_counter()
        run(steps)
        el = time.perf_counter() - t0
        per = [int(ctx.device_stats(d)["chunks"]) for d in range(nd)]
        kms = [round(ctx.device_stats(d)["kernel_ms"] / max(1, steps), 3) for d in range(nd)]
    finally:
        ctx.close()
    return {"n_devices": nd, "value": round(n * nd * steps / el, 1), "ms_per_step": round(el / steps * 1e3, 4),
            "catalogs_per_step": n * nd, "chunks_per_device": per, "kernel_ms_per_step_per_device": kms,
            "jobs_in_flight": depth,
            "note": "one process, dp_create(n_devices=%d) (the cgo shim's topology, INTEGRATION.md): one "
                    "submitting thread and host pool per device; not value" % nd}


def output_bytes(res) -> int:
    """Every output word the kernel writes: a 32-byte result
    record per problem (status, flags, core length and offset, steps, BCP
    bytes), the installed bitmaps, the core identities."""
    n = len(res["status"])
    return n * 32 + 4 * int(res["inst_off"][-1]) + 4 * int(res["core_len"].sum())


def class_mix(res) -> dict:
    """A / B / UNSAT-BCP / UNSAT-search / budget (dp_flag bits)."""
    st, fl = res["status"], res["flags"]
    sat, unsat = st == 1, st == -1
    return {"sat": int(sat.sum()), "unsat": int(unsat.sum()), "incomplete": int((st == 0).sum()),
            "error": int((st == -2).sum()),
            "class_a": int((sat & ((fl & 2) == 0)).sum()), "class_b": int((sat & ((fl & 2) != 0)).sum()),
            "unsat_bcp": int((unsat & ((fl & 16) != 0)).sum()),
            "unsat_search": int((unsat & ((fl & 16) == 0)).sum()),
            "budget": int(((fl & 64) != 0).sum())}


KEYS = ("status", "flags", "installed", "core_len", "steps")


def same_results(a, b) -> bool:
    if not all(np.array_equal(a[k], b[k]) for k in KEYS):
        return False
    for p in np.flatnonzero(a["core_len"]):
        c0, c1 = int(a["core_off"][p]), int(a["core_off"][p]) + int(a["core_len"][p])
        if not np.array_equal(a["core"][c0:c1], b["core"][c0:c1]):
            return False
    return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--inproc", action="store_true",
                    help="one process drives the N GPUs (dp_create(n_devices=N), the cgo shim's topology) "
                         "instead of one torchrun rank per GPU")
    ap.add_argument("--no-inproc-leg", action="store_true",
                    help="torchrun runs with N > 1: skip the one-process leg after the timed region")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--problems", type=int, default=0,
                    help="catalogs per step and rank (weak) or in total (strong); 0: WORKLOADS")
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--depth", type=int, default=0,
                    help="host-to-host jobs in flight; 0: enough to give every pipeline lane a chunk")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--kernel-steps", type=int, default=20,
                    help="steps of the device-resident (kernel-only) secondary figure; 0: skip")
    ap.add_argument("--record-form", choices=("packed", "p16d", "u16", "i32"), default="packed",
                    help="the records the GPU legs are given: dp_lower_into NARROW|PACKED (P8D/P16D/P16, "
                         "default), NARROW|PACKED|NO_P8 (P16D/P16: A/B), NARROW (U16) or int32 (staged by the host)")
    ap.add_argument("--e2e-steps", type=int, default=10,
                    help="steps of the lowering-inclusive (wire -> results) secondary figure; 0: skip")
    ap.add_argument("--kernel-depth", type=int, default=0,
                    help="kernel-only batches in flight; 0: one per pipeline lane (dp_lanes)")
    ap.add_argument("--kernel-only", action="store_true",
                    help="skip the host-to-host leg (profiling runs of the solve kernel)")
    ap.add_argument("--flags", type=int, default=0,
                    help="dp_opts.flags (diagnostic placements: 1 group, 2 HBM, 4 mid groups)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r06_pmc_traffic.jsonl"),
                    help="HBM bytes per solve kernel dispatch from separate rocprofv3 --pmc passes; "
                         "used for roofline.traffic when its config/problems match")
    ap.add_argument("--sq-json", default=os.path.join(ROOT, "profiles", "r06_sq_split.json"),
                    help="SQ instruction counts per wave of this build (scripts/pmc_sq_r02.sh + sq_summary.py), "
                         "for roofline.issue")
    args = ap.parse_args()
    maybe_relaunch(args)

    from deppy_amd import _lib, shard  # noqa: E402  (after the relaunch decision)

    g = shard.init_from_env("nccl")
    rank, world, local = g.rank, g.world, g.local
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    wl = WORKLOADS[args.config]
    nd = args.gpus if args.inproc else 1  # devices this process drives
    if args.scaling == "weak":
        n = (args.problems or wl[0]) * nd
        first = shard.shard_seed(args.seed, rank, n)
    else:
        total = args.problems or wl[1]
        lo, hi = shard.strong_range(total, rank, world)
        n, first = hi - lo, args.seed + lo
    lw, lw32, t_lower, wa = lowered_config(args.config, n, first, args.record_form)
    ctx = _lib.Context(0 if nd > 1 else local, nd, flags=args.flags)
    global LANES
    LANES = ctx.lanes()

    # host-to-host: depth jobs in flight, each the whole batch.  The pipeline
    # has LANES chunk slots per device (dp_lanes: two per lane stream, one
    # stream per hardware queue); by default as many jobs are in flight as
    # fill them.
    depth = args.depth
    if depth <= 0 and not args.kernel_only:  # (profiling runs count solve dispatches: none extra)
        ctx.stats(reset=True)
        ctx.submit(lw.rec_off, lw.rec).wait()
        depth = max(1, LANES // max(1, ctx.stats(reset=True)["chunks"]))
    outs = [_lib.result_arrays(lw.rec_off, lw.rec) for _ in range(depth)]

    def run_steps(k):
        jobs = []
        for i in range(k):
            if len(jobs) == depth:
                jobs.pop(0).wait()
            jobs.append(ctx.submit(lw.rec_off, lw.rec, outs[i % depth]))
        for j in jobs:
            j.wait()

    if args.kernel_only:  # profiling: only the device-resident leg below
        args.steps = 1
        st, elapsed, res, deterministic = ctx.stats(), float("inf"), None, None
        per_device = None
    else:
        run_steps(max(args.warmup, 1))
        first_res = ctx.submit(lw.rec_off, lw.rec).wait()  # cold-free single call, for the check
        g.barrier()
        ctx.stats(reset=True)
        t0 = time.perf_counter()
        run_steps(args.steps)
        t1 = time.perf_counter()
        g.barrier()
        per_device = [int(ctx.device_stats(d)["chunks"]) for d in range(nd)]
        st = ctx.stats(reset=True)
        elapsed = g.max(t1 - t0)
        res = ctx.submit(lw.rec_off, lw.rec).wait()
        deterministic = same_results(res, first_res) and all(
            same_results(res, {**o, "status": o["status"][:n], "flags": o["flags"][:n],
                               "core_len": o["core_len"][:n], "steps": o["steps"][:n]}) for o in outs)

    value = world * n * args.steps / elapsed if args.scaling == "weak" else \
        (args.problems or wl[1]) * args.steps / elapsed
    chunks = max(st["chunks"], 1)
    step_s = elapsed / args.steps
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "resolutions/s",
        "n_gpus": world * nd,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": wl[2] % (n // nd), "catalogs_per_step_per_gpu": n // nd,
                   "record_forms": record_forms(lw),
                   "placements": {k: v // max(args.steps, 1) for k, v in st["placed"].items() if v},
                   "placement_launches": {k: v // max(args.steps, 1) for k, v in st["placed_launches"].items() if v},
                   "parallelism": ("dp%d (host partition; one process, dp_create(n_devices=%d))" % (nd, nd)
                                   if nd > 1 else "dp%d (host partition; one process per GPU)" % world),
                   "n_devices_per_process": nd, "chunks_per_device_timed": per_device, "seed": args.seed,
                   "path": "host memory -> host memory (dp_submit/dp_job_wait), %d jobs in flight" % depth},
        "pipeline": {"chunks_per_step": round(chunks / args.steps, 2),
                     "kernel_ms_per_chunk": round(st["kernel_ms"] / chunks, 4),
                     "note": "chunk kernels share the GPU with the other chunks in flight"},
        "pcie": {"h2d_GBs": round(st["h2d_bytes"] / (elapsed if world == 1 else step_s * args.steps) / 1e9, 2),
                 "d2h_GBs": round(st["d2h_bytes"] / (elapsed if world == 1 else step_s * args.steps) / 1e9, 2),
                 "h2d_bytes_per_step": st["h2d_bytes"] // args.steps, "peak_GBs": PCIE_PEAK_GBS},
        "host_ms_per_step": {k: round(st[k] / args.steps, 4) for k in ("stage_ms", "plan_ms", "wait_ms", "scatter_ms")},
        "allocs_in_timed_region": int(st["allocs"]),
        "direct_chunks_per_step": round(st["direct_chunks"] / args.steps, 2),
        "bcp": {"visited_bytes_per_resolution": round(st["bcp_bytes"] / max(st["problems"], 1), 1)
                if st["bcp_bytes"] else None,
                "GBs": round(st["bcp_bytes"] / elapsed / 1e9, 2) if elapsed != float("inf") and st["bcp_bytes"]
                else None,
                "note": "bytes unit propagation reads (watch entries, row offsets, literals, values; in LDS "
                        "for one-wavefront problems, HBM for multi-wave), counted in the kernel (dp_stats); "
                        "null: not counted (the register-capped one-wavefront build, used for small "
                        "footprints, leaves the counter out to stay spill-free)"},
        "records_pinned": bool(lw.pinned),
        "classes": class_mix(res) if res is not None else None,
        "deterministic": bool(deterministic),
        "build": _lib.build_info(),
        "host_lowering_res_per_s": round(n / t_lower, 1),
        "host_lowering_note": "dp_lower_into (packed 16-bit records, storage reused) on the host pool; not in value",
    }
    if not args.kernel_only and args.e2e_steps > 0:
        line["end_to_end"] = {
            "res_per_s": round(end_to_end(ctx, wa, n, args.e2e_steps), 1),
            "steps": args.e2e_steps,
            "note": "wire format -> dp_lower_into -> dp_submit/dp_job_wait -> results, 2 batches in flight "
                    "(lowering of batch i+1 overlaps the solve of batch i); what BenchmarkSolve times "
                    "(NewSolver(WithInput)+Solve, bench_test.go:66-77); not value"}
        try:  # (a leg beside value: its failure must not cost the line)
            line["end_to_end_device"] = end_to_end_device(ctx, wa, lw, n, args.e2e_steps)
        except Exception as e:  # noqa: BLE001
            line["end_to_end_device"] = {"res_per_s": None, "error": repr(e)}
        line["solve_batch_api"] = {
            "res_per_s": round(solve_batch_api(ctx, wa, n, max(2, args.e2e_steps // 2)), 1),
            "steps": max(2, args.e2e_steps // 2),
            "note": "deppy_amd.sat.solve_wire (SolveBatch from the wire format to host results, as the cgo "
                    "shim calls the library): dp_lower_into NARROW|PACKED|PINNED into reused storage + dp_solve, "
                    "one batch at a time; not value"}
        try:
            line["solve_batch_api"]["device_lowering_res_per_s"] = round(
                solve_batch_api_device(ctx, wa, n, max(2, args.e2e_steps // 2)), 1)
        except Exception as e:  # noqa: BLE001
            line["solve_batch_api"]["device_lowering_res_per_s"] = None
            line["solve_batch_api"]["device_lowering_error"] = repr(e)
        line["solve_batch_api"]["device_lowering_note"] = (
            "the same from the compact wire (sat.solve_wire on a Wire32Arrays: dp_lower_device + dp_solve)")

    if args.kernel_steps > 0:
        # the solve kernel alone, records resident in HBM (dp_upload): serial
        # launches give the per-launch device time the roofline uses (HIP
        # events on the launch's stream; rocprofv3 --kernel-trace of
        # `bench.py --kernel-only` reports the same kernels), then one batch
        # per pipeline lane in flight gives the rate the kernel sustains
        kdepth = args.kernel_depth or LANES
        slots = [ctx.upload(lw.rec_off, lw.rec) for _ in range(1 if args.kernel_only else kdepth)]
        slots[0].run()
        kms = []
        for _ in range(args.kernel_steps):
            slots[0].run()
            kms.append(ctx.last_kernel_ms())
        tk = float("nan")
        # whole rounds of kdepth launches: a partial last round would run its
        # few launches with the GPU mostly idle (config 4: each launch is a
        # persistent grid of 256 catalogs)
        ksteps = -(-args.kernel_steps // kdepth) * kdepth
        if not args.kernel_only:  # (profiling runs keep every launch serial)
            for s_ in slots:
                s_.run()
            t0 = time.perf_counter()
            for i in range(ksteps):
                s_ = slots[i % kdepth]
                if i >= kdepth:
                    s_.wait()
                s_.launch()
            for s_ in slots:
                s_.wait()
            tk = time.perf_counter() - t0
        kres = slots[0].download()
        for s_ in slots:
            s_.free()
        if res is None:
            res = kres
            line["classes"] = class_mix(res)
        rec_bytes, _ = _lib.device_bytes(lw.rec_off, lw.rec)
        alg = rec_bytes + output_bytes(kres)
        k_ms = float(np.mean(kms))
        achieved = alg / (k_ms * 1e-3) / 1e9
        line["kernel_only"] = {"res_per_s": round(n * ksteps / tk, 1),
                               "ms_per_step": round(tk / ksteps * 1e3, 4),
                               "steps": ksteps,
                               "serial_launch_ms": round(k_ms, 4),
                               "identical_to_host_path": bool(same_results(kres, res)) if res is not None else None,
                               "batches_in_flight": kdepth,
                               "note": "records resident in HBM, %d batches in flight; not value" % kdepth}
        traffic = None
        if args.pmc_json and os.path.exists(args.pmc_json):
            with open(args.pmc_json) as f:
                for ln in f:
                    pmc = json.loads(ln)
                    if pmc.get("config") == args.config and pmc.get("problems") == n:
                        traffic = pmc.get("hbm_bytes_per_dispatch")
        line["roofline"] = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                            "kernel": "solve_kernel (one launch of the batch, serial, records in HBM)",
                            "kernel_ms": round(k_ms, 4), "algorithmic_bytes_per_launch": int(alg),
                            "traffic_over_algorithmic": round(traffic / alg, 3) if traffic else None,
                            "issue": issue_roofline(args.sq_json, args.config,
                                                    n * ksteps / tk if tk == tk else None)}
        # the same bytes at the sustained rate: batches in flight, records resident
        # (algorithmic bytes per batch / kernel_only.ms_per_step)
        sus = alg / (tk / ksteps) / 1e9 if tk == tk else None  # (--kernel-only keeps launches serial)
        line["roofline"]["sustained"] = None if sus is None else {
            "achieved": round(sus, 3), "frac": round(sus / HBM_PEAK_GBS, 6), "ms_per_batch": round(tk / ksteps * 1e3, 4),
            "note": "algorithmic bytes / kernel_only.ms_per_step (%d batches in flight)" % kdepth}

    if rank == 0 and not args.no_cpu:
        from oracle import oracle  # CPU baseline + checker only
        share = cpu_share()
        threads = share["cores"]
        o = oracle.solve_batch(lw32.rec_off, lw32.rec, 0, threads)  # also the parity check
        ok = same_results(res, o)
        # latency: single catalogs alone, host to host, beside one oracle thread
        lat_g, lat_c = [], []
        for p in range(min(n, 20)):
            a, b = int(lw.rec_off[p]), int(lw.rec_off[p + 1])
            one_off = np.array([0, b - a], np.int64)
            one = np.ascontiguousarray(lw.rec[a:b])
            ctx.solve(one_off, one)
            t0 = time.perf_counter()
            ctx.solve(one_off, one)
            lat_g.append(time.perf_counter() - t0)
            a, b = int(lw32.rec_off[p]), int(lw32.rec_off[p + 1])
            one_off = np.array([0, b - a], np.int64)
            one = np.ascontiguousarray(lw32.rec[a:b])
            t0 = time.perf_counter()
            oracle.solve_batch(one_off, one, 0, 1)
            lat_c.append(time.perf_counter() - t0)
        # the same catalogs without the call overheads: the kernel of one
        # catalog resident in HBM, and one oracle thread's solve inside a batch
        lat_k = []
        for p in range(min(n, 20)):
            a, b = int(lw.rec_off[p]), int(lw.rec_off[p + 1])
            r1 = ctx.upload(np.array([0, b - a], np.int64), np.ascontiguousarray(lw.rec[a:b]))
            r1.run()
            r1.run()
            lat_k.append(ctx.last_kernel_ms())
            r1.free()
        m = min(n, 20)
        sub_off = np.ascontiguousarray(lw32.rec_off[:m + 1])
        sub = np.ascontiguousarray(lw32.rec[:int(sub_off[-1])])
        reps, t0 = 0, time.perf_counter()
        while reps < 3 or time.perf_counter() - t0 < 0.5:
            oracle.solve_batch(sub_off, sub, 0, 1)
            reps += 1
        cpu_in_batch_ms = (time.perf_counter() - t0) / reps / m * 1e3
        line["latency"] = {"gpu_ms_median": round(float(np.median(lat_g)) * 1e3, 3),
                           "cpu_1thread_ms_median": round(float(np.median(lat_c)) * 1e3, 3),
                           "gpu_ms_p90": round(float(np.percentile(lat_g, 90)) * 1e3, 3),
                           "cpu_1thread_ms_p90": round(float(np.percentile(lat_c, 90)) * 1e3, 3),
                           "gpu_kernel_ms_median": round(float(np.median(lat_k)), 4),
                           "cpu_1thread_in_batch_ms_per_catalog": round(cpu_in_batch_ms, 4),
                           "catalogs": len(lat_g),
                           "note": "one catalog alone, host to host (dp_solve: the latency path for small "
                                   "batches of one-wavefront problems; one oracle thread beside it). Both "
                                   "medians include the Python wrapper's per-call overhead; "
                                   "gpu_kernel_ms_median is the catalog's kernel alone (resident in HBM) "
                                   "and cpu_1thread_in_batch_ms_per_catalog one oracle thread's solve "
                                   "without a call around it"}
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.solve_batch(lw32.rec_off, lw32.rec, 0, threads)
            reps += 1
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        cpu_t = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": round(reps * n / cpu_t, 1), "unit": "resolutions/s",
                                "cores": threads, "kind": "port",
                                "node_cores": threads * world,
                                "node_value_linear": round(reps * n / cpu_t * world, 1),
                                "sample": "the timed batch (%d catalogs) solved %d times by "
                                          "oracle/sat_oracle.c, one solver thread per core (%.1f s); "
                                          "nproc %s, affinity %d, cgroup quota %s; node_cores = this share "
                                          "x %d ranks (each rank's share), node_value_linear = value x ranks"
                                          % (n, reps, cpu_t, share["nproc"], share["affinity"],
                                             share["cgroup_quota"], world)}
        if "end_to_end" in line:
            line["end_to_end"]["cpu_res_per_s"] = round(cpu_end_to_end(wa, lw32, n, threads, 3.0), 1)
            line["end_to_end"]["cpu_note"] = ("dp_lower_into to int32 records + oracle/sat_oracle.c, %d threads "
                                              "(the lowering is the product's C++; the reference lowers in Go)"
                                              % threads)
        line["verified_bit_exact_vs_oracle"] = bool(ok)
        line["verified_note"] = "GPU on the packed 16-bit records vs oracle on the int32 records, every field incl. cores"
    if world > 1 and not args.no_inproc_leg and args.scaling == "weak" and not args.kernel_only:
        # the shipped one-process topology on the same node, after the timed
        # region: rank 0 drives all N GPUs while the other ranks wait
        g.barrier()
        if rank == 0:
            line["inproc"] = inproc_leg(args.config, n, world, args.seed, args.steps, args.warmup,
                                        args.record_form)
        g.barrier()
    if rank == 0:
        print(json.dumps(line), flush=True)
    g.close()


if __name__ == "__main__":
    main()
