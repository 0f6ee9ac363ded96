"""Summarise scripts/pmc_fetch_split.sh: per config, the solve kernel's
L2-to-fabric reads by request size, their destinations, its writes, the
SQC's instruction / scalar-data requests and the L2 hit rate, per run of the
batch (bench.py --kernel-only runs the batch K + 1 times).

Bytes: 32 B, 64 B and 128 B read requests at their sizes (gfx950 has a
counter per size; FETCH_SIZE tallies every request that is not 32 B at 64 B,
which is why MI355X_MICROARCH.md doubles it for wide streaming reads).

usage: python scripts/fetch_split.py <out_dir>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
out = {}
for err in sorted(glob.glob(root + "/c*_size.err")):
    cfg = os.path.basename(err)[1:].split("_")[0]
    agg = defaultdict(float)
    for d in glob.glob("%s/c%s_*" % (root, cfg)):
        if not os.path.isdir(d):
            continue
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "solve_kernel" in r["Kernel_Name"]:
                    agg[r["Counter_Name"]] += float(r["Counter_Value"])
    line = {}
    try:
        txt = open("%s/c%s_size.json" % (root, cfg)).read().strip().splitlines()
        line = json.loads([t for t in txt if t.startswith("{")][-1])
    except (OSError, IndexError, ValueError):
        pass
    runs = (7 if cfg != "4" else 3)
    g = lambda k: agg.get(k, 0.0) / runs  # noqa: E731
    rd_bytes = 32 * g("TCC_EA0_RDREQ_32B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + 128 * g("TCC_EA0_RDREQ_128B_sum")
    wr_bytes = 32 * (g("TCC_EA0_WRREQ_sum") - g("TCC_EA0_WRREQ_64B_sum")) + 64 * g("TCC_EA0_WRREQ_64B_sum")
    alg = (line.get("roofline") or {}).get("algorithmic_bytes_per_launch")
    out[cfg] = {
        "problems": (line.get("config") or {}).get("catalogs_per_step_per_gpu"),
        "algorithmic_bytes_per_run": alg,
        "read_requests": {"all": g("TCC_EA0_RDREQ_sum"), "32B": g("TCC_EA0_RDREQ_32B_sum"),
                          "64B": g("TCC_EA0_RDREQ_64B_sum"), "128B": g("TCC_EA0_RDREQ_128B_sum"),
                          "dram": g("TCC_EA0_RDREQ_DRAM_sum"), "dram_32B": g("TCC_EA0_RDREQ_DRAM_32B_sum"),
                          "io_32B": g("TCC_EA0_RDREQ_IO_32B_sum"), "uncached_32B": g("TCC_EA0_RD_UNCACHED_32B_sum")},
        "read_bytes_by_size": round(rd_bytes),
        "fetch_size_x2_bytes": round(2 * 64 * (g("TCC_EA0_RDREQ_sum") - g("TCC_EA0_RDREQ_32B_sum"))
                                     + 2 * 32 * g("TCC_EA0_RDREQ_32B_sum")),
        "write_requests": {"all": g("TCC_EA0_WRREQ_sum"), "64B": g("TCC_EA0_WRREQ_64B_sum"),
                           "io_32B": g("TCC_EA0_WRREQ_WRITE_IO_32B_sum"), "dram": g("TCC_EA0_WRREQ_DRAM_sum")},
        "write_bytes": round(wr_bytes),
        "traffic_over_algorithmic": round((rd_bytes + wr_bytes) / alg, 3) if alg else None,
        "sqc": {"inst_req": g("SQC_TC_INST_REQ"), "data_read_req": g("SQC_TC_DATA_READ_REQ"),
                "icache_misses": g("SQC_ICACHE_MISSES"), "dcache_misses": g("SQC_DCACHE_MISSES")},
        "l2": {"req": g("TCC_REQ_sum"), "read": g("TCC_READ_sum"), "hit": g("TCC_HIT_sum"), "miss": g("TCC_MISS_sum"),
               "hit_rate": round(g("TCC_HIT_sum") / max(1.0, g("TCC_HIT_sum") + g("TCC_MISS_sum")), 4)},
        "runs": runs,
    }
print(json.dumps(out, indent=1))
