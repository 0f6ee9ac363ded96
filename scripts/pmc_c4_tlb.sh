#!/bin/bash
# Config 4 under load: UTCL1 translation hits/misses and L2 hit/miss (two
# separate PMC passes of the solve kernel, 256 catalogs).
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_c4
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --output-format csv -d gpurun_out/pmc_c4/tlb -o run -- python3 scripts/config4.py 256 1 > gpurun_out/pmc_c4/tlb.out 2> gpurun_out/pmc_c4/tlb.err || { tail -5 gpurun_out/pmc_c4/tlb.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_c4/l2 -o run -- python3 scripts/config4.py 256 1 > gpurun_out/pmc_c4/l2.out 2> gpurun_out/pmc_c4/l2.err || { tail -5 gpurun_out/pmc_c4/l2.err; exit 1; }
python3 - <<'PY'
import csv, glob
for d in ("tlb", "l2"):
    tot = {}
    for f in glob.glob("gpurun_out/pmc_c4/%s/**/*counter_collection.csv" % d, recursive=True):
        for r in csv.DictReader(open(f)):
            if "solve_kernel" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print(d, tot)
PY
