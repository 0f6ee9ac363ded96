"""Benchmark: batched pkg/sat resolution on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]

One step = one pass of the solve kernel over one batch of BASELINE config 2:
10,000 synthetic operator catalogs (~200 bundle entities, Dependency +
Conflict + AtMost; SURVEY.md §8(d) generator), resident in HBM when the timed
region starts.  Steps are pipelined `--depth` deep (default 3) as a serving
loop would run them: the batch is resident in `depth` slots, step i launches
slot i % depth (dp_launch) after waiting for that slot's previous step
(dp_wait), so one step's tail of hard catalogs overlaps the next step's bulk.
Every step still resolves its whole batch; `serial_ms_per_step` reports the
unpipelined launch+wait time beside it.  With N > 1 (torchrun, one process per GPU) every rank solves
its own 10,000 catalogs (distinct seeds): weak scaling, no collective on the
data path (torch.distributed is used only for the barrier and the max-over-
ranks of the timing).

Rank 0 prints one JSON line.  `value` = resolutions/s over all ranks.
`roofline.achieved` = compulsory bytes of the batch (input records + outputs,
DESIGN.md §Measurement) / the solve kernel's mean device time (HIP events on
its stream).  `cpu_baseline` = the CPU restatement (oracle/, "port") on the
host, on the same batch repeated for a bounded time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from deppy_amd import _lib, shard  # noqa: E402

METRIC = "resolutions/sec (node) on synthetic catalogs at 1/2/4/8 GPUs; BCP HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


# BASELINE.json configs as bench workloads: (default catalogs per GPU, description)
WORKLOADS = {
    2: (10000, "config2: %d synthetic operator catalogs per GPU (P=40 packages, ~240 variables; "
               "Dependency+Conflict+AtMost), one wavefront per catalog"),
    3: (125000, "config3: %d small catalogs per GPU (P~U{4..12}, ~20-70 variables; 1M over 8 GPUs "
                "by host partition), one wavefront per catalog"),
    4: (256, "config4: %d OLM-scale catalogs per GPU (P=5000, ~55k variables, deep dependency "
             "chains), one 8-wave workgroup per catalog"),
    5: (10000, "config5: %d mixed-size catalogs per GPU (P~U{4..400}, 50%% with injected "
               "infeasibility), UNSAT-heavy"),
}


def lowered_config(config, n, seed):
    w = _lib.generate(config, n, seed)
    wa = _lib.WireArrays(**{k: w[k] for k in (
        "prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off", "con_arg",
        "str_off")}, str_bytes=w["str_bytes"].tobytes())
    t0 = time.perf_counter()
    lw = _lib.Lowered(wa)
    t_lower = time.perf_counter() - t0
    return lw, t_lower


def compulsory_bytes(lw, res) -> int:
    """Input records + every output word the kernel writes.
    Records count in their device form: LDS-path problems are stored in
    16-bit form (2 bytes per word after the int32 header; "B/2-equivalents
    when int16 literals are used"), the others at 4 bytes per word."""
    rec_bytes, _ = _lib.device_bytes(lw.rec_off, lw.rec)
    n = lw.n
    out = n * (1 + 4 + 4 + 8)  # status, flags, core_len, steps
    out += 4 * int(res["inst_off"][-1])  # installed bitmaps
    out += 4 * int(res["core_len"].sum())  # cores
    return rec_bytes + out


def _same(a, b) -> bool:
    return all(np.array_equal(a[k], b[k]) for k in ("status", "flags", "installed", "core_len", "core", "steps"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--problems", type=int, default=0,
                    help="catalogs per GPU (0: the config's default, WORKLOADS)")
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--depth", type=int, default=8,
                    help="steps in flight (1 = launch+wait per step); 8 = two per hardware queue")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic_config2.json"),
                    help="HBM bytes per solve run measured by separate rocprofv3 --pmc passes "
                         "(scripts/gpu_check.sh); used for roofline.traffic on the config it was taken on")
    args = ap.parse_args()
    if args.problems <= 0:
        args.problems = WORKLOADS[args.config][0]

    g = shard.init_from_env("nccl")
    rank, world, local = g.rank, g.world, g.local

    lw, t_lower = lowered_config(args.config, args.problems, shard.shard_seed(args.seed, rank, args.problems))
    ctx = _lib.Context(local, 1)

    # PCIe-inclusive single pass (host records -> host results), reported only
    t0 = time.perf_counter()
    ctx.solve(lw.rec_off, lw.rec)
    t_pcie = time.perf_counter() - t0

    depth = max(1, args.depth)
    slots = [ctx.upload(lw.rec_off, lw.rec) for _ in range(depth)]

    def steps(n, kms):
        for i in range(n):
            r = slots[i % depth]
            if i >= depth:
                r.wait()
                kms.append(ctx.last_kernel_ms())
            r.launch()
        for i in range(max(0, n - depth), n):
            slots[i % depth].wait()
            kms.append(ctx.last_kernel_ms())

    # unpipelined reference figure (not the metric): launch + wait per step
    serial = []
    for _ in range(3):
        t0 = time.perf_counter()
        slots[0].run()
        serial.append(time.perf_counter() - t0)

    steps(args.warmup, [])
    g.barrier()
    kms = []
    t0 = time.perf_counter()
    steps(args.steps, kms)
    t1 = time.perf_counter()
    g.barrier()
    elapsed = g.max(t1 - t0)
    res = slots[0].download()
    same = all(_same(res, x.download()) for x in slots[1:])
    for x in slots:
        x.free()

    value = shard.aggregate_rate(args.problems, world, args.steps, elapsed)
    st = res["status"]
    kernel_ms = float(np.mean(kms))
    nbytes = compulsory_bytes(lw, res)
    achieved = nbytes / (kernel_ms * 1e-3) / 1e9

    traffic = None
    if args.pmc_json and os.path.exists(args.pmc_json):
        with open(args.pmc_json) as f:
            pmc = json.load(f)
        if pmc.get("config") == args.config and pmc.get("problems") == args.problems:
            traffic = pmc.get("hbm_bytes_per_dispatch")

    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "resolutions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": WORKLOADS[args.config][1] % args.problems,
                   "catalogs_per_gpu": args.problems, "parallelism": "dp%d (host partition)" % world,
                   "seed": args.seed},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                     "traffic": traffic, "kernel_ms": round(kernel_ms, 4),
                     "algorithmic_bytes_per_launch": nbytes,
                     "effective_GBs_per_step": round(nbytes / (elapsed / args.steps) / 1e9, 3)},
        "pipeline_depth": depth,
        "serial_ms_per_step": round(float(np.median(serial)) * 1e3, 4),
        "slots_identical": bool(same),
        "classes": {"sat": int((st == 1).sum()), "unsat": int((st == -1).sum()),
                    "incomplete": int((st == 0).sum()), "error": int((st == -2).sum()),
                    "class_b": int(((res["flags"] & 2) != 0).sum())},
        "pcie_inclusive_res_per_s": round(args.problems / t_pcie, 1),
        "host_lowering_res_per_s": round(args.problems / t_lower, 1),
    }

    if rank == 0 and not args.no_cpu:
        from oracle import oracle  # CPU baseline + checker only
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        o = oracle.solve_batch(lw.rec_off, lw.rec, 0, threads)  # also the parity check
        ok = (np.array_equal(o["status"], st) and np.array_equal(o["flags"], res["flags"])
              and np.array_equal(o["installed"], res["installed"])
              and np.array_equal(o["core_len"], res["core_len"])
              and np.array_equal(o["steps"], res["steps"]))
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.solve_batch(lw.rec_off, lw.rec, 0, threads)
            reps += 1
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        cpu_t = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": round(reps * args.problems / cpu_t, 1),
                                "unit": "resolutions/s", "cores": threads, "kind": "port",
                                "sample": "the timed batch (%d catalogs) solved %d times by "
                                          "oracle/sat_oracle.c on %d host threads (%.1f s)"
                                          % (args.problems, reps, threads, cpu_t)}
        line["verified_bit_exact_vs_oracle"] = bool(ok)
    if rank == 0:
        print(json.dumps(line), flush=True)
    g.close()


if __name__ == "__main__":
    main()
