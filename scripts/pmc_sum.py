"""Sum rocprofv3 --pmc counters of the solve kernel's dispatches.

usage: python scripts/pmc_sum.py <pmc_dir> [<pmc_dir> ...]  -> JSON {counter: total}
"""
import csv
import glob
import json
import sys

tot = {}
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "solve_kernel" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print(json.dumps(tot))
