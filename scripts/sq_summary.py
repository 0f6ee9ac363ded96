"""Summarise scripts/pmc_sq_r02.sh output: per-wave cycle split and
instruction mix of the solve kernel (SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_*
count quad-cycles on gfx950, MI355X_MICROARCH.md)."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq"
out = {}
for d in sorted(glob.glob(root + "/c*_a")):
    cfg = d.split("/")[-1][1:].split("_")[0]
    agg = defaultdict(float)
    for part in ("a", "b"):
        for f in glob.glob("%s/c%s_%s/**/*counter_collection.csv" % (root, cfg, part), recursive=True):
            for r in csv.DictReader(open(f)):
                if "solve_kernel" in r["Kernel_Name"]:
                    agg[r["Counter_Name"]] += float(r["Counter_Value"])
    waves = agg["SQ_WAVES"]
    wc = agg["SQ_WAVE_CYCLES"]
    out[cfg] = {
        "waves": waves,
        "active_frac": round(agg["SQ_ACTIVE_INST_ANY"] / wc, 3),
        "wait_any_frac": round(agg["SQ_WAIT_ANY"] / wc, 3),
        "wait_inst_frac": round(agg["SQ_WAIT_INST_ANY"] / wc, 3),
        "wave_cycles_per_wave": round(4 * wc / waves),
        "per_wave": {k: round(agg[k] / waves, 1) for k in (
            "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
            "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH")},
        "active_valu_frac": round(agg["SQ_ACTIVE_INST_VALU"] / wc, 3),
        "active_lds_frac": round(agg["SQ_ACTIVE_INST_LDS"] / wc, 3),
        "wait_inst_lds_frac": round(agg["SQ_WAIT_INST_LDS"] / wc, 3),
    }
# the library the counters came from (bench.py uses them only for that build)
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from deppy_amd import _lib  # noqa: E402
out["build"] = _lib.build_info()
print(json.dumps(out, indent=1))
